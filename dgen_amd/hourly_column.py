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
    background thread; a cell is the agent's row (a READ-ONLY float64 ndarray
    view: the plane is shared; assigning cells through the frame gives the
    column its own copy), and only reading a cell waits for the plane;
  * yearly: the [n][51] host array and each agent's list length; a cell is a
    fresh Python list of the agent's N + 1 values, made when it is read.
Slicing, take, groupby, merge and concat move indices (concat of columns
over different planes keeps a list of segments, no dense copy); pickling (the
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


class _Segments:
    """Columns of different planes concatenated without copying them
    (pd.concat of size_chunk frames, reference dgen_model.py:384): row j of
    the virtual [n][w] array is row idx_k[j - off_k] of segment k's plane, cut
    to that segment's cell length.  result() (a dense, zero-padded copy) is
    built only when the whole 2-D array is asked for."""

    def __init__(self, parts):
        # parts: (plane, idx, lens-or-None, lists) of each concatenated column
        self.parts = [(p, np.asarray(i, np.int64), None if ln is None else np.asarray(ln, np.int64))
                      for p, i, ln, _ in parts]
        self.off = np.concatenate([[0], np.cumsum([i.shape[0] for _, i, _ in self.parts])]).astype(np.int64)
        self.n = int(self.off[-1])
        self._dense = None

    def row(self, j):
        k = int(np.searchsorted(self.off, j, side="right") - 1)
        p, idx, ln = self.parts[k]
        r = idx[j - self.off[k]]
        a = p.result()
        return a[r] if ln is None else a[r, :ln[r]]

    def done(self) -> bool:
        return all(p.done() for p, _, _ in self.parts)

    def result(self) -> np.ndarray:
        if self._dense is None:
            rows = [p.result()[i] for p, i, _ in self.parts]
            w = max((r.shape[1] for r in rows), default=0)
            self._dense = np.concatenate([r if r.shape[1] == w else np.pad(r, ((0, 0), (0, w - r.shape[1])))
                                          for r in rows]) if rows else np.zeros((0, 0))
        return self._dense

    def lens(self) -> np.ndarray:
        out = []
        for p, i, ln in self.parts:
            out.append(ln[i] if ln is not None else np.full(i.shape[0], p.result().shape[1], np.int64))
        return np.concatenate(out) if out else np.zeros(0, np.int64)


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
        return None if isinstance(self._plane, _Segments) else self._plane.result()

    def _cell(self, a, j):
        """Cell j: a read-only float64 view of the agent's row (the planes are
        shared by every reader: writing through a cell would change the
        others' data -- assign with df.at / __setitem__, which gives the
        column its own copy), or a new list (yearly cells)."""
        if isinstance(self._plane, _Segments):
            r = self._plane.row(j)
        else:
            r = a[j] if self._lens is None else a[j, :self._lens[j]]
        if self._lists:
            return r.tolist()
        r = r.view()
        r.flags.writeable = False
        return r

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
        if self._lists and self._lens is not None and a is not None:
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
        if isinstance(self._plane, _Segments) or not self._plane.done():
            return len(self) * NH * 8
        return len(self) * self._rows().shape[1] * 8

    def __setitem__(self, key, value):
        """Assign cells (df.at[...] = ..., or the array API): the column first takes its own copy
        of its rows, so the shared plane and the other columns over it are
        unchanged.  value: one cell (applied to every selected row) or one cell
        per selected row."""
        a = np.array(self.to_2d(), dtype=np.float64, copy=True)
        lens = self._cell_lens().copy()
        pos = np.arange(len(self))[key]
        pos = np.atleast_1d(pos)
        one = np.ndim(value) <= 1 and not (len(pos) > 1 and np.ndim(value) == 1 and
                                          len(value) == len(pos) and np.ndim(value[0]) >= 1)
        cells = [value] * len(pos) if one else list(value)
        if len(cells) != len(pos):
            raise ValueError("one cell per selected row expected")
        for k, v in zip(pos.tolist(), cells):
            r = np.asarray(v, dtype=np.float64).ravel()
            if r.shape[0] > a.shape[1]:
                a = np.pad(a, ((0, 0), (0, r.shape[0] - a.shape[1])))
            a[k, :r.shape[0]] = r
            a[k, r.shape[0]:] = 0.0
            lens[k] = r.shape[0]
        self._plane = _Ready(a)
        self._idx = np.arange(a.shape[0], dtype=np.int64)
        full = (lens == a.shape[1]).all() and not self._lists
        self._lens = None if full else lens

    def isna(self) -> np.ndarray:
        return np.zeros(len(self), dtype=bool)

    def take(self, indices, allow_fill=False, fill_value=None):
        ix = np.asarray(indices, dtype=np.int64)
        if allow_fill and (ix < 0).any():
            if (ix < -1).any():
                raise ValueError("invalid take index")
            # missing rows (reindex): NaN series of the full width, materialised
            a = self._plane.result()
            if isinstance(self._plane, _Segments):
                src = RowColumn(_Ready(a), self._idx, self._plane.lens(), self._lists)
                return src.take(indices, allow_fill=allow_fill, fill_value=fill_value)
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
        # different planes (each chunk's own): O(1), the rows stay where they are
        parts = []
        for c in to_concat:
            if isinstance(c._plane, _Segments) and c._idx.shape[0] == c._plane.n and \
                    (c._idx == np.arange(c._plane.n)).all():
                parts.extend((p, i, ln, c._lists) for p, i, ln in c._plane.parts)
            elif isinstance(c._plane, _Segments):     # a selection of a concatenation
                for j in c._idx.tolist():
                    k = int(np.searchsorted(c._plane.off, j, side="right") - 1)
                    p, idx, ln = c._plane.parts[k]
                    parts.append((p, idx[j - c._plane.off[k]:j - c._plane.off[k] + 1], ln, c._lists))
            else:
                parts.append((c._plane, c._idx, c._lens, c._lists))
        seg = _Segments(parts)
        return cls(seg, None, None, all(c._lists for c in to_concat))

    def _cell_lens(self) -> np.ndarray:
        if isinstance(self._plane, _Segments):
            return self._plane.lens()[self._idx]
        if self._lens is None:
            w = getattr(self._plane, "width", None)          # a DevicePlane: no download for its width
            return np.full(len(self), w if w is not None else self._rows().shape[1], dtype=np.int64)
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
        a = self._plane.result()
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
