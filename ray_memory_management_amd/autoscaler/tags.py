"""Node tags. Parity: reference python/ray/autoscaler/tags.py."""
TAG_RAY_NODE_KIND = "ray-node-type"
TAG_RAY_USER_NODE_TYPE = "ray-user-node-type"
TAG_RAY_NODE_STATUS = "ray-node-status"
TAG_RAY_LAUNCH_CONFIG = "ray-launch-config"

NODE_KIND_HEAD = "head"
NODE_KIND_WORKER = "worker"
NODE_KIND_UNMANAGED = "unmanaged"

STATUS_UNINITIALIZED = "uninitialized"
STATUS_UP_TO_DATE = "up-to-date"
STATUS_UPDATE_FAILED = "update-failed"
