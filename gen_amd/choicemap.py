"""A minimal choice map for the observation side of the PF boundary.

Gen's `choicemap((:chain => t => :y, y_t))` (src/choice_map.jl:659-670) maps
hierarchical addresses to values.  Here an address is a tuple, e.g.
("chain", 3, "y") for `:chain => 3 => :y`; `choicemap(((addr), value), ...)`
builds one.  Only what the hot path consumes is implemented: lookup by the
address of one time step (the flat `to_array` idea, choice_map.jl:163-169).
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

    def __repr__(self):
        return f"ChoiceMap({self._d!r})"


def choicemap(*pairs) -> ChoiceMap:
    cm = ChoiceMap()
    for addr, value in pairs:
        cm[addr] = value
    return cm


EmptyChoiceMap = ChoiceMap
