class RayServeException(Exception):
    pass
