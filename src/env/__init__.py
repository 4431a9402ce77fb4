"""Vectorised GPU traffic environment (the home the reference left empty:
src/env/__init__.py and src/env/traffic_env.py are 0 bytes upstream)."""
from .traffic_env import TrafficEnv, EnvConfig  # noqa: F401
