"""Python-side helpers for gob values (the Go types a net/rpc call carries).

Go structs travel as named structs: pass a dataclass (its class name is the Go
type name, its fields in declaration order are the Go fields) or a ``GoStruct``.
Decoded structs come back as ``GoStruct`` objects with attribute access.
"""
from __future__ import annotations


class GoUint(int):
    """A Go ``uint`` (gob encodes int and uint differently)."""

    def __gob_value__(self):
        return ("uint", int(self))


class GoSlice(list):
    """A typed Go slice (needed only for an empty slice of a non-int type)."""

    def __init__(self, items=(), proto=0):
        super().__init__(items)
        self.proto = proto

    def __gob_value__(self):
        return ("slice", list(self), self.proto)


class GoStruct:
    """A Go struct value: ``GoStruct("Args", [("A", 7), ("B", 8)])`` or keywords."""

    def __init__(self, type_name: str, fields=None, **kw):
        object.__setattr__(self, "_name", type_name)
        items = list(fields.items()) if isinstance(fields, dict) else list(fields or [])
        items += list(kw.items())
        object.__setattr__(self, "_fields", items)

    def __gob_value__(self):
        return ("struct", self._name, self._fields)

    @property
    def type_name(self) -> str:
        return self._name

    def fields(self):
        return list(self._fields)

    def __getattr__(self, k):
        for n, v in object.__getattribute__(self, "_fields"):
            if n == k:
                return v
        raise AttributeError(k)

    def __getitem__(self, k):
        return self.__getattr__(k)

    def __eq__(self, o):
        if isinstance(o, GoStruct):
            return self._name == o._name and self._fields == o._fields
        return NotImplemented

    def __repr__(self):
        inner = ", ".join(f"{k}={v!r}" for k, v in self._fields)
        return f"{self._name or 'struct'}({inner})"
