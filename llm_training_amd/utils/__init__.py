from .imports import import_object, normalize_path
from .misc import ContextManagers, StrEnum, copy_method_signature

__all__ = ["import_object", "normalize_path", "ContextManagers", "StrEnum", "copy_method_signature"]
