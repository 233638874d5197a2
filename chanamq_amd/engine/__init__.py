"""Data plane: GPU (HIP) step engine, golden Python model, control tables, traffic."""
from .control import ControlError, ControlState, DEFAULT_VHOST, entity_id, normalize_vhost
