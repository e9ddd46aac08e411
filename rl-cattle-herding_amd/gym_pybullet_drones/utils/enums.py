"""Enums with the reference's names and values (reference: utils/enums.py)."""
from cattleherd.spaces import ActionType, DroneModel, ImageType, ObservationType, Physics  # noqa: F401
