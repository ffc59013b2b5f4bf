"""Per-agent series columns built in O(1) (size_frame's default "lazy" mode).

The reference fills list cells per agent: three 8760-h series
(`financial_functions.py:523-539`) and seven yearly lists (cash flow, energy
value, bills: `:449-474`, `:505-521`).  Its consumers read the hourly cells
with len() and np.asarray (`attachment_rate_functions.py:166-182`), the yearly
ones as lists (`finance_series_export.py:51-64` writes an agent's records only
when its cells are lists), and drop them before writing agent outputs
(`dgen_model.py:441-458`).

Here such a column is a pandas ExtensionArray over one [n][w] float64 array
and an index of its rows, so building it costs nothing per agent:
  * hourly: the array is an engine.HostPlane still crossing PCIe on a
    background thread; a cell is the agent's row (a float64 ndarray view),
    and only reading a cell waits for the plane;
  * yearly: the [n][51] host array and each agent's list length; a cell is a
    fresh Python list of the agent's N + 1 values, made when it is read.
Slicing, take, groupby, merge and concat move indices; pickling (the
reference returns size_chunk's frame from a pool worker) ships the rows."""
from __future__ import annotations

import numpy as np
from pandas.api.extensions import ExtensionArray, ExtensionDtype, register_extension_dtype

NH = 8760


class _Ready:
    """An array already on the host (the HostPlane interface)."""

    __slots__ = ("_a", "n")

    def __init__(self, a: np.ndarray):
        self._a = a
        self.n = a.shape[0]

    def result(self) -> np.ndarray:
        return self._a

    def done(self) -> bool:
        return True


@register_extension_dtype
class RowDtype(ExtensionDtype):
    name = "dgen_rows"
    type = object
    kind = "O"
    na_value = None

    @classmethod
    def construct_array_type(cls):
        return RowColumn


class RowColumn(ExtensionArray):
    """Rows `idx` of an [n][w] array (a HostPlane or a host array).  lens:
    per-row cell lengths (None: the full row); lists: cells are Python lists
    (else float64 ndarray views)."""

    def __init__(self, plane, idx=None, lens=None, lists: bool = False):
        self._plane = plane
        self._idx = (np.arange(plane.n, dtype=np.int64) if idx is None
                     else np.asarray(idx, dtype=np.int64))
        self._lens = None if lens is None else np.asarray(lens, dtype=np.int64)
        self._lists = bool(lists)

    def _like(self, idx):
        return RowColumn(self._plane, idx, self._lens, self._lists)

    # -- construction ------------------------------------------------------
    @classmethod
    def _from_sequence(cls, scalars, *, dtype=None, copy=False):
        if isinstance(scalars, RowColumn):
            return scalars.copy() if copy else scalars
        cells = list(scalars)
        lists = bool(cells) and all(isinstance(c, list) for c in cells)
        rows = [np.asarray(c, dtype=np.float64).ravel() for c in cells]
        lens = np.array([r.shape[0] for r in rows], dtype=np.int64)
        w = int(lens.max()) if rows else 0
        a = np.zeros((len(rows), w))
        for k, r in enumerate(rows):
            a[k, :r.shape[0]] = r
        full = bool(rows) and (lens == w).all() and not lists
        return cls(_Ready(a), None, None if full else lens, lists)

    @classmethod
    def _from_factorized(cls, values, original):
        raise NotImplementedError("series columns are not factorizable")

    # -- the array protocol ------------------------------------------------
    @property
    def dtype(self):
        return RowDtype()

    def __len__(self) -> int:
        return int(self._idx.shape[0])

    def _rows(self) -> np.ndarray:
        return self._plane.result()

    def _cell(self, a, j):
        r = a[j] if self._lens is None else a[j, :self._lens[j]]
        return r.tolist() if self._lists else r

    def __getitem__(self, item):
        if isinstance(item, (int, np.integer)):
            return self._cell(self._rows(), self._idx[item])
        if isinstance(item, tuple) and len(item) == 1:
            item = item[0]
        if isinstance(item, slice):
            return self._like(self._idx[item])
        key = np.asarray(item)
        if key.dtype == bool:
            return self._like(self._idx[key])
        return self._like(self._idx[key.astype(np.int64)])

    def __iter__(self):
        a = self._rows()
        for j in self._idx:
            yield self._cell(a, j)

    def __array__(self, dtype=None, copy=None):
        a = self._rows()
        out = np.empty(len(self), dtype=object)
        if self._lists and self._lens is not None:
            # lists grouped by length: one tolist per group
            ln = self._lens[self._idx]
            for w in np.unique(ln):
                ks = np.nonzero(ln == w)[0]
                vals = a[self._idx[ks], :w].tolist()
                for k, v in zip(ks.tolist(), vals):
                    out[k] = v
            return out
        for k, j in enumerate(self._idx):
            out[k] = self._cell(a, j)
        return out

    @property
    def nbytes(self) -> int:
        return len(self) * (self._rows().shape[1] if self._plane.done() else NH) * 8

    def isna(self) -> np.ndarray:
        return np.zeros(len(self), dtype=bool)

    def take(self, indices, allow_fill=False, fill_value=None):
        ix = np.asarray(indices, dtype=np.int64)
        if allow_fill and (ix < 0).any():
            if (ix < -1).any():
                raise ValueError("invalid take index")
            # missing rows (reindex): NaN series of the full width, materialised
            a = self._rows()
            rows = np.full((ix.shape[0], a.shape[1]), np.nan)
            ok = ix >= 0
            rows[ok] = a[self._idx[ix[ok]]]
            lens = None
            if self._lens is not None:
                lens = np.full(ix.shape[0], a.shape[1], dtype=np.int64)
                lens[ok] = self._lens[self._idx[ix[ok]]]
            return RowColumn(_Ready(rows), None, lens, self._lists)
        return self._like(self._idx[ix])

    def copy(self):
        return self._like(self._idx.copy())

    @classmethod
    def _concat_same_type(cls, to_concat):
        to_concat = list(to_concat)
        c0 = to_concat[0]
        if all(c._plane is c0._plane and c._lists == c0._lists for c in to_concat):
            return cls(c0._plane, np.concatenate([c._idx for c in to_concat]), c0._lens, c0._lists)
        parts = [c.to_2d() for c in to_concat]
        w = max(p.shape[1] for p in parts)
        rows = np.concatenate([np.pad(p, ((0, 0), (0, w - p.shape[1]))) for p in parts])
        lens = np.concatenate([c._cell_lens() for c in to_concat])
        full = (lens == w).all() and not c0._lists
        return cls(_Ready(rows), None, None if full else lens, all(c._lists for c in to_concat))

    def _cell_lens(self) -> np.ndarray:
        if self._lens is None:
            return np.full(len(self), self._rows().shape[1], dtype=np.int64)
        return self._lens[self._idx]

    def cell_lens(self) -> np.ndarray:
        """Each cell's length (the row width where no lengths are kept)."""
        return self._cell_lens()

    def cells_are_lists(self) -> bool:
        """True when cells read as Python lists (the reference's yearly cells)."""
        return self._lists

    def ready(self) -> bool:
        """True once the rows are on the host (reading a cell will not wait)."""
        return self._plane.done()

    def to_2d(self) -> np.ndarray:
        """The column's rows as one [len][w] float64 array (waits; entries past
        a cell's length are whatever the source holds there)."""
        a = self._rows()
        if self._idx.shape[0] == a.shape[0] and (self._idx == np.arange(a.shape[0])).all():
            return a
        return a[self._idx]

    def __getstate__(self):
        return {"rows": self.to_2d(), "lens": None if self._lens is None else self._cell_lens(),
                "lists": self._lists}

    def __setstate__(self, st):
        self._plane = _Ready(st["rows"])
        self._idx = np.arange(st["rows"].shape[0], dtype=np.int64)
        self._lens = st["lens"]
        self._lists = st["lists"]

    def _formatter(self, boxed=False):
        return lambda v: f"<{len(v)} values>"

    def __repr__(self):
        state = "on host" if self.ready() else "downloading"
        kind = "lists" if self._lists else "arrays"
        return f"<RowColumn: {len(self)} agents, {kind}, {state}>"


def hourly_column(plane) -> RowColumn:
    """An hourly column over a HostPlane (cells: float64 row views)."""
    return RowColumn(plane)


def yearly_column(a: np.ndarray, lens) -> RowColumn:
    """A yearly column over a host [n][w] array (cells: lists of lens[i] values)."""
    return RowColumn(_Ready(np.asarray(a, dtype=np.float64)), None, lens, lists=True)
