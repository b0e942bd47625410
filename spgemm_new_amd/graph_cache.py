"""Per-graph cache of ``MaxKGraph`` objects.

The reference rebuilt its kernel objects and re-read the .warp4 file on every
autograd call (utils/models.py:78-86, spmm_maxk.cu:117).  Here the schedule is
built once per (indptr, indices, values) storage and reused while the tensors
are unchanged (storage pointer, size and in-place version counter).
"""
from __future__ import annotations

from collections import OrderedDict

from .ops import MaxKGraph

_CACHE: "OrderedDict[tuple, MaxKGraph]" = OrderedDict()
_MAX = 8


def _key(t):
    return (t.data_ptr(), t.numel(), t._version, str(t.device))


def graph_for(indptr, indices, values=None, **kw) -> MaxKGraph:
    key = (_key(indptr), _key(indices), None if values is None else _key(values),
           tuple(sorted(kw.items())))
    g = _CACHE.get(key)
    if g is None:
        g = MaxKGraph(indptr, indices, values, **kw)
        _CACHE[key] = g
        while len(_CACHE) > _MAX:
            _CACHE.popitem(last=False)
    else:
        _CACHE.move_to_end(key)
    return g


def clear():
    _CACHE.clear()
