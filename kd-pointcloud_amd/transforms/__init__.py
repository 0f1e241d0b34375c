from .transforms import *  # noqa: F401,F403
