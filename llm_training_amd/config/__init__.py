from .loader import deep_merge, expand_dotted, instantiate, load_config

__all__ = ["deep_merge", "expand_dotted", "instantiate", "load_config"]
