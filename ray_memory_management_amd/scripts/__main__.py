import sys

from ray_memory_management_amd.scripts.scripts import main

sys.exit(main())
