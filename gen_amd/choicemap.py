"""A minimal choice map for the observation side of the PF boundary.

Gen's `choicemap((:chain => t => :y, y_t))` (src/choice_map.jl:659-670) maps
hierarchical addresses to values.  Here an address is a tuple, e.g.
("chain", 3, "y") for `:chain => 3 => :y`; `choicemap(((addr), value), ...)`
builds one.  Besides lookup by address, `to_array` / `from_array` flatten a
choice map's values and rebuild one of the same address structure
(choice_map.jl:163-225).
"""
from __future__ import annotations


def _norm(addr):
    if isinstance(addr, tuple):
        return addr
    if isinstance(addr, list):
        return tuple(addr)
    return (addr,)


class ChoiceMap:
    def __init__(self, items=None):
        self._d = {}
        for a, v in (items or {}).items() if isinstance(items, dict) else (items or []):
            self[a] = v

    def __setitem__(self, addr, value):
        self._d[_norm(addr)] = value

    def __getitem__(self, addr):
        return self._d[_norm(addr)]

    def has_value(self, addr) -> bool:
        return _norm(addr) in self._d

    def get(self, addr, default=None):
        return self._d.get(_norm(addr), default)

    def __contains__(self, addr):
        return self.has_value(addr)

    def __len__(self):
        return len(self._d)

    def __iter__(self):
        return iter(self._d.items())

    def isempty(self) -> bool:
        return not self._d

    def merge(self, other: "ChoiceMap") -> "ChoiceMap":
        """merge (choice_map.jl:237-266): error on overlapping addresses."""
        out = ChoiceMap(dict(self._d))
        for a, v in other:
            if a in out._d:
                raise ValueError(f"merge: both choice maps have a value at {a}")
            out._d[a] = v
        return out

    def to_array(self):
        """to_array(choices, Float64) (choice_map.jl:163-169): every value in
        address order (the order the choices were added), vectors flattened."""
        import numpy as np

        parts = [np.atleast_1d(np.asarray(v, dtype=np.float64)).ravel() for v in self._d.values()]
        return np.concatenate(parts) if parts else np.zeros(0)

    def from_array(self, arr) -> "ChoiceMap":
        """from_array(proto_choices, arr) (choice_map.jl:190-225): a choice map
        with this one's addresses and value shapes, values read off arr in
        to_array's order.  It is an error if arr has the wrong length."""
        import numpy as np

        arr = np.asarray(arr, dtype=np.float64).ravel()
        out, pos = ChoiceMap(), 0
        for a, v in self._d.items():
            shape = np.shape(v)
            size = int(np.prod(shape)) if shape else 1
            if pos + size > arr.size:
                raise ValueError("from_array: the array is shorter than the prototype's values")
            chunk = arr[pos:pos + size]
            out._d[a] = float(chunk[0]) if not shape else chunk.reshape(shape).copy()
            pos += size
        if pos != arr.size:
            raise ValueError("from_array: the array is longer than the prototype's values")
        return out

    def __repr__(self):
        return f"ChoiceMap({self._d!r})"


def choicemap(*pairs) -> ChoiceMap:
    cm = ChoiceMap()
    for addr, value in pairs:
        cm[addr] = value
    return cm


EmptyChoiceMap = ChoiceMap


class Selection:
    """A set of addresses (src/address.jl:54,352 `select(addrs...)`), with the
    same tuple convention as ChoiceMap: select("slope") names :slope,
    select(("chain", 3, "x")) names :chain => 3 => :x."""

    def __init__(self, addrs=()):
        self.addrs = frozenset(_norm(a) for a in addrs)

    def __contains__(self, addr):
        return _norm(addr) in self.addrs

    def __iter__(self):
        return iter(self.addrs)

    def __len__(self):
        return len(self.addrs)

    def __repr__(self):
        return f"select({', '.join(map(repr, sorted(self.addrs, key=repr)))})"


def select(*addrs) -> Selection:
    return Selection(addrs)
