import sys

from ray_memory_management_amd.rllib.scripts import main

sys.exit(main())
