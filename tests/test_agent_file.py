"""Agent-file ingestion (input_data_functions.py:387-446): state filter, ISO
regions, the empty-region error, Parquet and pickle forms."""
import pandas as pd
import pytest

from dgen_amd.agent_file import read_agent_file


def _frame():
    return pd.DataFrame({"agent_id": [1, 2, 3, 4], "state_abbr": ["DE", "CA", "DE", "NY"],
                         "load_kwh_per_customer_in_bin": [9e3, 1.2e4, 8e3, 1.1e4]})


@pytest.mark.parametrize("ext", [".pkl", ".parquet"])
def test_state_filter_and_iso_region(tmp_path, ext):
    p = str(tmp_path / f"agents{ext}")
    (_frame().to_pickle if ext == ".pkl" else _frame().to_parquet)(p)
    df = read_agent_file(p, state_to_model=["DE"], region="DE")
    assert list(df["agent_id"]) == [1, 3]
    assert len(read_agent_file(p, state_to_model=["DE"], region="NYISO")) == 4
    with pytest.raises(ValueError, match="Region not present"):
        read_agent_file(p, state_to_model=["TX"], region="TX")


def test_rejects_other_files(tmp_path):
    p = tmp_path / "agents.csv"
    _frame().to_csv(p)
    with pytest.raises(ValueError):
        read_agent_file(str(p))
