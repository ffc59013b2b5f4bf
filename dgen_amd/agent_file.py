"""Pre-generated agent files (SURVEY 8f-3 ingestion).

Restates the file half of ``input_data_functions.import_agent_file``
(dgen_os/python/input_data_functions.py:387-446): read the scenario's agent
table from ``<input_agent_dir>/<name>.pkl``, keep the states being modelled
unless the region is one of the ISO regions, and refuse an empty result with
the reference's message.  The frame then goes through ``size_chunk`` /
``PopulationBuilder`` (columnar.py), which compiles each distinct tariff once
and uploads the agent columns to the device.

The reference's tariff reassignment (``elec.reassign_agent_tariffs``, a DB
query) is out of scope: agents keep the ``tariff_dict`` the file holds.
Only agent files the user's own pipeline wrote are read here; Parquet is
accepted too (same columns, no pickle involved).
"""
from __future__ import annotations

import os
from typing import Iterable, Optional

import pandas as pd

ISO_LIST = ["ERCOT", "NEISO", "NYISO", "CAISO", "PJM", "MISO", "SPP"]   # input_data_functions.py:424


def read_agent_file(path: str, state_to_model: Optional[Iterable[str]] = None,
                    region: Optional[str] = None) -> pd.DataFrame:
    """The agent DataFrame of a pre-generated agent file (.pkl or .parquet).

    state_to_model: the scenario's states (``scenario_settings.state_to_model``);
    region: ``scenario_settings.region`` -- ISO regions keep every row
    (input_data_functions.py:433-437)."""
    ext = os.path.splitext(path)[1].lower()
    if ext == ".parquet":
        df = pd.read_parquet(path)
    elif ext in (".pkl", ".pickle"):
        df = pd.read_pickle(path)
    else:
        raise ValueError(f"unsupported agent file type {ext!r} (expected .pkl or .parquet)")
    if not isinstance(df, pd.DataFrame):
        raise TypeError(f"{path}: expected a pandas DataFrame, got {type(df).__name__}")
    if region not in ISO_LIST and state_to_model is not None:
        df = df[df["state_abbr"].isin(list(state_to_model))]
    if df.empty:
        raise ValueError("Region not present within pre-generated agent file - Edit Inputsheet")
    return df
