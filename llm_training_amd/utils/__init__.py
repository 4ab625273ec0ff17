from .imports import import_object, normalize_path

__all__ = ["import_object", "normalize_path"]
