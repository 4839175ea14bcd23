from . import mnist  # noqa: F401
