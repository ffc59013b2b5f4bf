"""Profile sources: what replaces the two per-agent SQL round trips of the
reference (agent_mutation/elec.py:508-558).

* ``ProfileStore``   in-memory tables keyed like the reference's SQL:
    load  <- (bldg_id, sector_abbr, state_abbr)  kwh_load_profile (8760)
    solar <- (solar_re_9809_gid, tilt, azimuth)  cf x 1e6 (8760 integers)
* ``SqlProfileSource`` runs the reference's own queries on a DB-API
  connection (psycopg2 / pg8000 / sqlite3) once per distinct key and caches the
  rows, so a chunk of agents costs one query per distinct profile, not two per
  agent.
"""
from __future__ import annotations

import json
from typing import Any, Dict, Hashable, List, Optional, Tuple

import numpy as np

NH = 8760


def load_key(agent) -> Tuple:
    return (agent["bldg_id"], agent["sector_abbr"], agent["state_abbr"])


def solar_key(agent) -> Tuple:
    return (agent["solar_re_9809_gid"], agent["tilt"], agent["azimuth"])


def _norm_key(k) -> Tuple:
    out = []
    for v in k:
        if isinstance(v, (np.integer,)):
            v = int(v)
        elif isinstance(v, (np.floating,)):
            v = float(v)
            if v.is_integer():
                v = int(v)
        elif isinstance(v, float) and v.is_integer():
            v = int(v)
        out.append(v)
    return tuple(out)


def _as_array(v) -> np.ndarray:
    if isinstance(v, str):
        v = json.loads(v)
    return np.asarray(v)


class ProfileStore:
    """Append-only profile tables with key -> row maps."""

    def __init__(self):
        self._shapes: List[np.ndarray] = []
        self._cfs: List[np.ndarray] = []
        self._lidx: Dict[Tuple, int] = {}
        self._sidx: Dict[Tuple, int] = {}
        self._stacked: Dict[str, Tuple[int, np.ndarray]] = {}

    # -- population -------------------------------------------------------
    def add_load(self, key, profile) -> int:
        k = _norm_key(key)
        if k in self._lidx:
            return self._lidx[k]
        a = np.asarray(profile, dtype=np.float32).ravel()
        if a.size != NH:
            raise ValueError(f"load profile {key} has {a.size} values, expected {NH}")
        self._lidx[k] = len(self._shapes)
        self._shapes.append(a)
        return self._lidx[k]

    def add_solar(self, key, cf_scaled) -> int:
        k = _norm_key(key)
        if k in self._sidx:
            return self._sidx[k]
        a = np.asarray(cf_scaled)
        if a.size != NH:
            raise ValueError(f"solar profile {key} has {a.size} values, expected {NH}")
        if not np.array_equal(a, np.round(a)):
            raise ValueError("solar cf must be the integer-scaled (x 1e6) DB values")
        self._sidx[k] = len(self._cfs)
        self._cfs.append(a.astype(np.int32).ravel())
        return self._sidx[k]

    @classmethod
    def from_arrays(cls, shapes, cfs, load_keys, solar_keys) -> "ProfileStore":
        st = cls()
        for k, row in zip(load_keys, shapes):
            st.add_load(k, row)
        for k, row in zip(solar_keys, cfs):
            st.add_solar(k, row)
        return st

    # -- lookup -----------------------------------------------------------
    def load_row(self, agent) -> int:
        k = _norm_key(load_key(agent))
        try:
            return self._lidx[k]
        except KeyError:
            raise KeyError(f"no load profile for (bldg_id, sector_abbr, state_abbr) = {k}") from None

    def solar_row(self, agent) -> int:
        k = _norm_key(solar_key(agent))
        try:
            return self._sidx[k]
        except KeyError:
            raise KeyError(f"no solar profile for (gid, tilt, azimuth) = {k}") from None

    def ensure(self, agents) -> None:
        """Hook for sources that fetch lazily (no-op for the in-memory store)."""

    def ensure_frame(self, df) -> None:
        """ensure() over an agent DataFrame (one fetch per distinct key)."""

    @property
    def n_load(self) -> int:
        return len(self._shapes)

    @property
    def n_solar(self) -> int:
        return len(self._cfs)

    def _stack(self, name: str, rows: List[np.ndarray], dtype) -> np.ndarray:
        hit = self._stacked.get(name)
        if hit is not None and hit[0] == len(rows):
            return hit[1]
        a = np.stack(rows) if rows else np.zeros((0, NH), dtype)
        self._stacked[name] = (len(rows), a)
        return a

    @property
    def shapes(self) -> np.ndarray:
        return self._stack("shapes", self._shapes, np.float32)

    @property
    def cfs(self) -> np.ndarray:
        return self._stack("cfs", self._cfs, np.int32)


class SqlProfileSource(ProfileStore):
    """Reference SQL (elec.py:514-519, 543-549) against a DB-API connection."""

    LOAD_SQL = ("SELECT bldg_id, sector_abbr, state_abbr, kwh_load_profile as consumption_hourly "
                "FROM diffusion_load_profiles.{sector_abbr}stock_load_profiles "
                "WHERE bldg_id = {bldg_id} AND sector_abbr = '{sector_abbr}' "
                "AND state_abbr = '{state_abbr}';")
    SOLAR_SQL = ("SELECT solar_re_9809_gid, tilt, azimuth, cf as generation_hourly, "
                 "1e6 as scale_offset FROM diffusion_resource_solar.solar_resource_hourly "
                 "WHERE solar_re_9809_gid = '{solar_re_9809_gid}' AND tilt = '{tilt}' "
                 "AND azimuth = '{azimuth}';")

    def __init__(self, con):
        super().__init__()
        self.con = con

    def _fetch(self, sql: str):
        cur = self.con.cursor()
        try:
            cur.execute(sql)
            row = cur.fetchone()
        finally:
            cur.close()
        return row

    def ensure_frame(self, df) -> None:
        cols = ["bldg_id", "sector_abbr", "state_abbr", "solar_re_9809_gid", "tilt", "azimuth"]
        uniq = df[cols].drop_duplicates()
        self.ensure([dict(zip(cols, r)) for r in uniq.itertuples(index=False, name=None)])

    def ensure(self, agents) -> None:
        for agent in agents:
            lk = _norm_key(load_key(agent))
            if lk not in self._lidx:
                sql = self.LOAD_SQL.format(bldg_id=lk[0], sector_abbr=lk[1], state_abbr=lk[2])
                row = self._fetch(sql)
                if row is None:
                    raise KeyError(f"no load profile row for {lk}")
                self.add_load(lk, _as_array(row[3]))
            sk = _norm_key(solar_key(agent))
            if sk not in self._sidx:
                sql = self.SOLAR_SQL.format(solar_re_9809_gid=sk[0], tilt=sk[1], azimuth=sk[2])
                row = self._fetch(sql)
                if row is None:
                    raise KeyError(f"no solar resource row for {sk}")
                self.add_solar(sk, _as_array(row[3]))


def as_source(con) -> ProfileStore:
    if isinstance(con, ProfileStore):
        return con
    if hasattr(con, "cursor"):
        return SqlProfileSource(con)
    raise TypeError("con must be a ProfileStore or a DB-API connection")
