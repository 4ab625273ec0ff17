"""Python front-end of the C++ packers (csrc/packing.cpp) with exact pure-Python equivalents used only
when the native library cannot be loaded (CPU-only environments without a build)."""
from __future__ import annotations

import torch


def _native():
    try:
        from ..ops.native import available, lib

        return lib() if available() else None
    except Exception:  # noqa: BLE001
        return None


def bfd_assign(lengths_sorted_desc: list[int], capacity: int) -> list[int]:
    """Bin index per item for best-fit over the given order (callers pass descending-length order)."""
    L = _native()
    if L is not None and lengths_sorted_desc:
        # the native op sorts stably by descending length itself: already-sorted input is unchanged
        return L.bfd_pack(torch.tensor(lengths_sorted_desc, dtype=torch.long), capacity).tolist()
    bins: list[int] = []
    out = []
    for n in lengths_sorted_desc:
        best, space = -1, None
        for j, rem in enumerate(bins):
            if rem >= n and (space is None or rem - n < space):
                best, space = j, rem - n
        if best < 0:
            bins.append(capacity - n)
            out.append(len(bins) - 1)
        else:
            bins[best] -= n
            out.append(best)
    return out


def group_by_length(lengths: list[int], max_length: int) -> list[list[int]]:
    """Groups of example indices (ascending length, greedy; reference instruction_tuning :102-121)."""
    if not lengths:
        return []
    L = _native()
    if L is not None:
        g = L.group_by_length(torch.tensor(lengths, dtype=torch.long), max_length).tolist()
    else:
        g = [0] * len(lengths)
        gi, s, c = 0, 0, 0
        for i in sorted(range(len(lengths)), key=lambda i: lengths[i]):
            n = lengths[i]
            if c == 0 or s + n + c <= max_length:
                s += n
                c += 1
            else:
                gi += 1
                s, c = n, 1
            g[i] = gi
    groups: dict[int, list[int]] = {}
    for i in sorted(range(len(lengths)), key=lambda i: lengths[i]):
        groups.setdefault(g[i], []).append(i)
    return [groups[k] for k in sorted(groups)]
