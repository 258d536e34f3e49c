"""Accelerator type constants for `@remote(accelerator_type=...)` (reference
python/ray/util/accelerators/accelerators.py lists NVIDIA parts; this framework targets AMD
Instinct GPUs). A node advertises ``accelerator_type:<name>`` as a custom resource."""
AMD_INSTINCT_MI355X = "AMD-Instinct-MI355X"
AMD_INSTINCT_MI350X = "AMD-Instinct-MI350X"
AMD_INSTINCT_MI325X = "AMD-Instinct-MI325X"
AMD_INSTINCT_MI300X = "AMD-Instinct-MI300X"
AMD_INSTINCT_MI250X = "AMD-Instinct-MI250X"


def detect_accelerator_type():
    """The AMD GPU model of device 0 (from torch's device name) or None."""
    try:
        import torch

        if torch.cuda.is_available():
            name = torch.cuda.get_device_name(0)
            for const in (AMD_INSTINCT_MI355X, AMD_INSTINCT_MI350X, AMD_INSTINCT_MI325X, AMD_INSTINCT_MI300X,
                          AMD_INSTINCT_MI250X):
                if const.split("-")[-1] in name:
                    return const
            return name
    except Exception:
        pass
    return None
