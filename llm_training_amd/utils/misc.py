"""Small utilities with the reference's names (src/llm_training/utils/context_managers.py:5-16,
decorators.py:9-21, str_enum.py:4-16)."""
from __future__ import annotations

import contextlib
import enum
import functools
from typing import Callable, ContextManager, Iterable


class ContextManagers(contextlib.AbstractContextManager):
    """Enter a list of context managers as one (exited in reverse order)."""

    def __init__(self, context_managers: Iterable[ContextManager]):
        self.context_managers = list(context_managers)
        self._stack: contextlib.ExitStack | None = None

    def __enter__(self):
        self._stack = contextlib.ExitStack()
        for cm in self.context_managers:
            self._stack.enter_context(cm)
        return self

    def __exit__(self, *exc):
        stack, self._stack = self._stack, None
        return stack.__exit__(*exc) if stack is not None else False


def copy_method_signature(ref_method: Callable, passthrough: bool = True):
    """Give ``method`` the signature/doc of ``ref_method``. With ``passthrough`` the decorated method
    body is replaced by a call to the same-named method of the next class in the MRO (used to expose
    a parent's signature on an override that only exists for typing)."""

    def decorator(method: Callable):
        if passthrough:
            def call_parent(self, *args, _mro_idx: int = 0, **kwargs):
                owner = type(self).mro()[_mro_idx]
                parent = getattr(super(owner, self), method.__name__)
                import inspect
                if "_mro_idx" in inspect.signature(parent, follow_wrapped=False).parameters:
                    kwargs["_mro_idx"] = _mro_idx + 1
                return parent(*args, **kwargs)
            fn = functools.update_wrapper(call_parent, method)
        else:
            fn = method
        fn.__signature__ = __import__("inspect").signature(ref_method)
        fn.__doc__ = ref_method.__doc__ or fn.__doc__
        return fn

    return decorator


class StrEnum(str, enum.Enum):
    """String-valued enum whose ``auto()`` values are the lower-cased member names."""

    def __new__(cls, value, *args, **kwargs):
        if not isinstance(value, str):
            raise TypeError(f"StrEnum values must be strings, got {type(value).__name__}: {value!r}")
        obj = str.__new__(cls, value)
        obj._value_ = value
        return obj

    def __str__(self) -> str:
        return str(self.value)

    @staticmethod
    def _generate_next_value_(name, start, count, last_values):
        return name.lower()
