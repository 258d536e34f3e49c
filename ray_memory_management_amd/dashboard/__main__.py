from ray_memory_management_amd.dashboard.head import main

main()
