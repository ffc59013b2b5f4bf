"""RowColumn (size_frame's default "lazy" series columns) under the pandas
operations the reference's consumers apply (attachment_rate_functions.py:
153-182: len per cell, np.asarray per row in iterrows; dgen_model.py:453 drop;
chunk frames concatenated, pickled from pool workers) -- CPU, with planes
that are already on the host and one that is still "downloading"."""
import pickle
import threading

import numpy as np
import pytest
import pandas as pd

from dgen_amd.hourly_column import NH, RowDtype, hourly_column, yearly_column


class _SlowPlane:
    """A HostPlane stand-in whose rows land when release() is called."""

    def __init__(self, a):
        self.n, self._a, self._ev = a.shape[0], a, threading.Event()

    def release(self):
        self._ev.set()

    def result(self):
        assert self._ev.wait(10), "plane never landed"
        return self._a

    def done(self):
        return self._ev.is_set()


def _frame(n=7, seed=0):
    rng = np.random.default_rng(seed)
    a, b = rng.random((n, NH)), rng.random((n, NH))
    pa, pb = _SlowPlane(a), _SlowPlane(b)
    df = pd.DataFrame({"agent_id": np.arange(n) + 100, "state": list("ABABCAB"[:n])})
    df["baseline_net_hourly"] = pd.Series(hourly_column(pa), index=df.index)
    df["adopter_net_hourly_pvonly"] = pd.Series(hourly_column(pb), index=df.index)
    df["adopter_net_hourly"] = df["adopter_net_hourly_pvonly"]
    return df, a, b, pa, pb


def test_building_and_dropping_do_not_wait():
    df, a, b, pa, pb = _frame()
    assert isinstance(df["baseline_net_hourly"].dtype, RowDtype)
    assert "downloading" in repr(df["baseline_net_hourly"].array)
    d2 = df.drop(columns=["adopter_net_hourly"]).copy()
    assert len(d2) == 7 and len(d2.iloc[2:5]) == 3 and not pa.done()
    pa.release(), pb.release()


def test_cells_are_the_rows():
    df, a, b, pa, pb = _frame()
    pa.release(), pb.release()
    for i, c in enumerate(df["baseline_net_hourly"]):
        assert isinstance(c, np.ndarray) and c.dtype == np.float64 and np.array_equal(c, a[i])
    assert np.array_equal(df["adopter_net_hourly"].iloc[3], b[3])
    assert (df["baseline_net_hourly"].map(len) == NH).all()
    for _, r in df.iterrows():
        assert np.array_equal(np.asarray(r["adopter_net_hourly_pvonly"], dtype=float), b[r["agent_id"] - 100])
    assert np.array_equal(df["baseline_net_hourly"].array.to_2d(), a)


def test_take_groupby_concat_pickle():
    df, a, b, pa, pb = _frame()
    pa.release(), pb.release()
    sub = df.iloc[[5, 1, 1]]
    assert [int(x) for x in sub["agent_id"]] == [105, 101, 101]
    assert np.array_equal(sub["baseline_net_hourly"].iloc[0], a[5])
    for s, g in df.groupby("state"):
        for _, r in g.iterrows():
            assert np.array_equal(r["baseline_net_hourly"], a[r["agent_id"] - 100])
    cat = pd.concat([df.iloc[:3], df.iloc[3:]], ignore_index=True)
    assert np.array_equal(cat["baseline_net_hourly"].array.to_2d(), a)
    other, a2, _, p2, q2 = _frame(seed=1)
    p2.release(), q2.release()
    cat2 = pd.concat([df, other], ignore_index=True)
    assert np.array_equal(cat2["baseline_net_hourly"].array.to_2d(), np.concatenate([a, a2]))
    back = pickle.loads(pickle.dumps(df.iloc[2:6]))
    assert np.array_equal(back["adopter_net_hourly"].array.to_2d(), b[2:6])
    re = df.reindex([0, 99])
    assert np.array_equal(re["baseline_net_hourly"].iloc[0], a[0]) and np.isnan(re["baseline_net_hourly"].iloc[1]).all()


def test_reading_waits_for_the_plane():
    df, a, b, pa, pb = _frame()
    got = []
    t = threading.Thread(target=lambda: got.append(np.asarray(df["baseline_net_hourly"].iloc[4])))
    t.start()
    t.join(0.2)
    assert t.is_alive() and not got          # still waiting
    pa.release()
    t.join(5)
    assert np.array_equal(got[0], a[4])
    pb.release()


def test_yearly_cells_are_lists_of_each_agents_length():
    """Yearly cells: Python lists of the agent's N + 1 values (what the
    reference's finance export requires, finance_series_export.py:51-64)."""
    rng = np.random.default_rng(3)
    a = rng.random((6, 51))
    n1 = np.array([26, 21, 26, 31, 51, 11])
    df = pd.DataFrame({"agent_id": np.arange(6), "s": list("ABABAB")})
    df["cash_flow"] = pd.Series(yearly_column(a, n1), index=df.index)
    for i, c in enumerate(df["cash_flow"]):
        assert isinstance(c, list) and c == a[i, :n1[i]].tolist()
    for _, r in df.iterrows():
        c = r.get("cash_flow")
        assert isinstance(c, list) and len(c) == n1[r["agent_id"]]
    assert df["cash_flow"].tolist()[3] == a[3, :31].tolist()
    g = pd.concat([df.iloc[4:], df.iloc[:2]], ignore_index=True)
    assert g["cash_flow"].iloc[0] == a[4].tolist() and g["cash_flow"].iloc[3] == a[1, :21].tolist()
    back = pickle.loads(pickle.dumps(df))
    assert [len(c) for c in back["cash_flow"]] == n1.tolist()
    m = df.merge(pd.DataFrame({"s": ["A", "B"], "rate": [1.0, 2.0]}), on="s", how="left")
    assert [c == a[k, :n1[k]].tolist() for k, c in zip(m["agent_id"], m["cash_flow"])] == [True] * 6


def test_mixed_concat_materialises():
    df, a, b, pa, pb = _frame()
    pa.release(), pb.release()
    y = pd.DataFrame({"baseline_net_hourly": pd.Series(yearly_column(np.ones((2, 5)), [5, 3]))})
    cat = pd.concat([df[["baseline_net_hourly"]], y], ignore_index=True)
    assert np.array_equal(np.asarray(cat["baseline_net_hourly"].iloc[0]), a[0])
    assert list(cat["baseline_net_hourly"].iloc[8]) == [1.0, 1.0, 1.0]


def test_cells_are_read_only_and_assignment_copies():
    """Hourly cells are views of a plane shared by every reader: writing
    through one fails; assigning through the frame gives the column its own
    rows and leaves the plane (and other columns over it) unchanged."""
    import pandas as pd
    from dgen_amd.hourly_column import RowColumn, _Ready
    a = np.arange(12, dtype=np.float64).reshape(3, 4)
    col = RowColumn(_Ready(a))
    other = RowColumn(_Ready(a))
    cell = col[1]
    with pytest.raises(ValueError):
        cell[0] = 99.0
    df = pd.DataFrame({"h": col, "g": other})
    df.at[1, "h"] = np.full(4, -1.0)           # as with the reference's object cells
    assert np.array_equal(np.asarray(df["h"].iloc[1]), np.full(4, -1.0))
    assert np.array_equal(a[1], [4.0, 5.0, 6.0, 7.0])            # the shared plane is untouched
    assert np.array_equal(np.asarray(df["g"].iloc[1]), [4.0, 5.0, 6.0, 7.0])


def test_concat_of_different_planes_keeps_segments():
    """pd.concat of chunk frames over different planes builds no dense copy:
    cells read through to each chunk's plane; the 2-D view is made on demand."""
    import pandas as pd
    from dgen_amd.hourly_column import RowColumn, _Ready, _Segments
    a = np.arange(8, dtype=np.float64).reshape(2, 4)
    b = 100 + np.arange(12, dtype=np.float64).reshape(3, 4)
    f = pd.concat([pd.DataFrame({"h": RowColumn(_Ready(a))}), pd.DataFrame({"h": RowColumn(_Ready(b))})],
                  ignore_index=True)
    col = f["h"].array
    assert isinstance(col._plane, _Segments) and col._plane._dense is None
    assert np.array_equal(np.asarray(f["h"].iloc[3]), b[1])
    assert col._plane._dense is None
    g = pd.concat([f, f.iloc[[0]]], ignore_index=True)
    assert np.array_equal(np.asarray(g["h"].iloc[5]), a[0])
    assert np.array_equal(g["h"].array.to_2d(), np.concatenate([a, b, a[:1]]))
    y1 = RowColumn(_Ready(np.ones((2, 5))), None, [3, 5], lists=True)
    y2 = RowColumn(_Ready(np.zeros((1, 2))), None, [2], lists=True)
    yc = RowColumn._concat_same_type([y1, y2])
    assert [len(c) for c in yc] == [3, 5, 2] and yc[2] == [0.0, 0.0]
