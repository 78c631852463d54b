"""Reporter constructs (``GetFluorFromPolPos.m:18-44``) as data instead of a file edit.

The reference hard-codes one construct and tells users to edit the file for others
(``README.md:33-34``, template at ``GetFluorFromPolPos.m:31-44``). Here a construct is a
value: gene length ``L0`` (``L = L0 + tau*v``, :19-20) and, per segment, the MS2/PP7 loop
start, end and loop count; multi-segment tables loop exactly as ``:47-70`` does.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Sequence

import numpy as np

from . import _lib


@dataclass
class Construct:
    L0: float
    ms2_start: Sequence[float]
    ms2_end: Sequence[float]
    ms2_loopn: Sequence[float]
    pp7_start: Sequence[float]
    pp7_end: Sequence[float]
    pp7_loopn: Sequence[float]
    name: str = field(default="custom")

    @property
    def n_seg(self) -> int:
        return len(self.ms2_start)

    def validate(self) -> None:
        n = self.n_seg
        arrs = [self.ms2_start, self.ms2_end, self.ms2_loopn, self.pp7_start, self.pp7_end, self.pp7_loopn]
        if not (1 <= n <= _lib.TCI_MAX_SEG) or any(len(a) != n for a in arrs):
            raise ValueError(f"construct needs 1..{_lib.TCI_MAX_SEG} segments, all tables the same length")
        for s in range(n):
            for a, e in ((self.ms2_start[s], self.ms2_end[s]), (self.pp7_start[s], self.pp7_end[s])):
                if not (0 <= a < e):
                    raise ValueError(f"segment {s}: need 0 <= start < end, got {a}, {e}")

    def to_c(self):
        """A ``tci_construct`` plus the arrays that keep its pointers alive."""
        self.validate()
        arrs = [np.ascontiguousarray(np.asarray(a, np.float64)) for a in
                (self.ms2_start, self.ms2_end, self.ms2_loopn, self.pp7_start, self.pp7_end, self.pp7_loopn)]
        cs = _lib.tci_construct(float(self.L0), self.n_seg, *[_lib.ptr(a, _lib._dp) for a in arrs])
        return cs, arrs


P2P_MS2V5_LACZ_PP7V4 = "P2P-MS2v5-LacZ-PP7v4"


def builtin_construct(name: str) -> Construct:
    """The constructs the reference defines. Only ``'P2P-MS2v5-LacZ-PP7v4'`` exists
    (``GetFluorFromPolPos.m:18-28``); any other name is an error, as in the reference."""
    if name == P2P_MS2V5_LACZ_PP7V4:
        return Construct(6.626, [0.024], [1.299], [24.0], [4.292], [5.758], [24.0], name)
    raise ValueError(f"construct {name!r} is not defined (GetFluorFromPolPos.m:18)")


def long_two_loop_construct() -> Construct:
    """2 stem-loop segments per dye on a 3x longer gene (19.878 kb)."""
    return Construct(19.878, [0.024, 6.650], [1.299, 7.925], [24.0, 24.0],
                     [12.912, 17.544], [14.378, 19.010], [24.0, 24.0], "2xloops-3xlength")


def as_construct(c) -> Construct:
    if isinstance(c, Construct):
        return c
    if isinstance(c, str):
        return builtin_construct(c)
    raise TypeError("construct must be a Construct or a construct name")
