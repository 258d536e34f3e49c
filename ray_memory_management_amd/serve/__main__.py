import sys

from ray_memory_management_amd.serve.scripts import main

sys.exit(main())
