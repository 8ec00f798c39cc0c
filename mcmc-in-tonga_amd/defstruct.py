"""Data and model types -- field-for-field mirror of DefStruct.jl.

``DataStruct`` (DefStruct.jl:5-30) keeps the reference's layout: ``rayX``,
``rayY``, ``rayZ``, ``U`` are m x n (points x rays, ray i = column i, NaN
tail padding) and ``rayL``/``rayU`` are (m-1) x n.  ``Model`` (DefStruct.jl:
32-48) is mutable, like the Julia ``mutable struct``.
"""
from dataclasses import dataclass, field
from typing import Optional

import numpy as np


@dataclass
class Ray:  # DefStruct.jl:1-3 (unused by the reference)
    x: np.ndarray
    y: np.ndarray
    z: np.ndarray


@dataclass
class DataStruct:  # DefStruct.jl:5-30
    tS: np.ndarray
    allaveatten: np.ndarray
    allLats: np.ndarray
    allLons: np.ndarray
    allSig: np.ndarray
    dataX: np.ndarray
    dataY: np.ndarray
    xVec: np.ndarray
    yVec: np.ndarray
    zVec: np.ndarray
    elonsX: np.ndarray
    elatsY: np.ndarray
    elons: np.ndarray
    elats: np.ndarray
    edep: np.ndarray
    coastX: np.ndarray
    coastY: np.ndarray
    rayX: np.ndarray
    rayY: np.ndarray
    rayZ: np.ndarray
    rayL: np.ndarray
    rayU: np.ndarray
    U: np.ndarray
    # device context cache (not a reference field): geometry is immutable
    _td_ctx: Optional[object] = field(default=None, repr=False, compare=False)


@dataclass
class Model:  # mutable struct Model, DefStruct.jl:32-48
    nCells: float
    xCell: np.ndarray
    yCell: np.ndarray
    zCell: np.ndarray
    zeta: np.ndarray
    phi: float = -1.0
    ptS: np.ndarray = field(default_factory=lambda: np.zeros(1))
    tS: np.ndarray = field(default_factory=lambda: np.zeros(1))
    likelihood: float = -1.0
    action: int = -1
    accept: int = -1
    zeta_xz: float = -1.0
    zeta_xy: float = -1.0

    def copy(self):
        """deepcopy(model) (TD_inversion_function.jl:84,130,186,224)."""
        return Model(float(self.nCells), self.xCell.copy(), self.yCell.copy(), self.zCell.copy(), self.zeta.copy(),
                     self.phi, np.array(self.ptS, copy=True), self.tS, self.likelihood, self.action, self.accept,
                     self.zeta_xz, self.zeta_xy)

    def cells(self):
        return (self.xCell, self.yCell, self.zCell, self.zeta)
