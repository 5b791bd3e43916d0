"""Compatibility module: code written against the reference's ``settings_dist``
(`settings_dist.py:1-42`) can ``from settings_dist import *`` unchanged."""
from unet_distributed_amd.settings import *  # noqa: F401,F403
