"""Engine._no_net_of (dgen_tables.no_net, ABI 12): a batch may run the
demand-charge kernels without their net-billing paths only when no agent can
reach a net-billing tariff -- initial tariff or any solar / storage rate-switch
candidate.  Host logic only (no GPU)."""
import numpy as np

from dgen_amd.engine import Engine
from dgen_amd.synth import make_population


class _Host(Engine):
    def __init__(self):          # no device: the batch logic only
        pass


def _eng(pop):
    e = _Host()
    e._tariff_mo = pop.tariffs["mo"].copy()
    e._switch_tariff = pop.switches["tariff"].copy()
    return e


def test_demand_charge_population_has_no_net_agent():
    pop = make_population("com_dc_batt", 3000)
    assert np.isin(pop.tariffs["mo"], (2, 3)).any()       # the table holds CA net-billing variants
    assert _eng(pop)._no_net_of(pop.cols, 3000)


def test_net_billing_agents_are_seen():
    pop = make_population("ca_res_storage", 3000)
    assert not _eng(pop)._no_net_of(pop.cols, 3000)


def test_switch_candidate_to_a_net_tariff_counts():
    pop = make_population("com_dc_batt", 2000)
    e = _eng(pop)
    cols = {k: np.asarray(v).copy() for k, v in pop.cols.items()}
    net_t = int(np.flatnonzero(np.isin(pop.tariffs["mo"], (2, 3)))[0])
    # one agent gets a storage-switch candidate that lands on a net tariff
    e._switch_tariff = np.concatenate([e._switch_tariff, [net_t]])
    cols["sw_storage_off"][7] = e._switch_tariff.size - 1
    cols["sw_storage_cnt"][7] = 1
    assert not e._no_net_of(cols, 2000)
    # an unknown switch table is conservative
    e._switch_tariff = None
    assert not e._no_net_of(pop.cols, 2000)


def test_nem_rows_are_the_leading_bins_only_run(monkeypatch):
    from dgen_amd.engine import profile_order
    pop = make_population("national_mixed", 3000)
    order = profile_order(pop.cols)
    cols = {k: np.asarray(v)[order] for k, v in pop.cols.items()}
    e = _eng(pop)
    k = e._nem_rows_of(cols, 3000)
    sl = cols["scratch_slot"]
    assert k > 0 and (sl[:k] < 0).all() and sl[k] >= 0
    monkeypatch.setenv("DGEN_NEM_SPLIT", "0")
    assert e._nem_rows_of(cols, 3000) == 0


class _Unconvertible:
    """Stands in for a device-tensor column (np.asarray raises)."""
    def __len__(self):
        return 3000

    def __array__(self, *a, **k):
        raise TypeError("can't convert cuda tensor to numpy")


def test_device_tensor_columns_keep_the_net_forms():
    pop = make_population("com_dc_batt", 3000)
    cols = dict(pop.cols)
    cols["tariff0"] = _Unconvertible()
    assert not _eng(pop)._no_net_of(cols, 3000)


class _Lib:
    def __init__(self):
        self.calls = []

    def __getattr__(self, name):
        def f(*a):
            self.calls.append((name, a[1:] if name.startswith("dgen_set") else ()))
            return 0
        return f


def test_tables_changed_after_upload_fall_back_to_general_forms():
    """no_net / nb_scan are decided at upload; a set_tariffs /
    set_switches before size() must not leave the NET = false kernels on."""
    from dgen_amd import _lib
    from dgen_amd.engine import AgentBatch
    e = _Host()
    e.lib, e.ctx, e.tables, e._tables_gen = _Lib(), None, _lib.Tables(), 5
    e.stream_handle = lambda: 0
    b = AgentBatch(n=10, n_scratch=4, cols={}, workspace=type("W", (), {"numel": lambda s: 8, "data_ptr": lambda s: 0})(),
                   c_agents=_lib.Agents(), nb_scan=False, no_net=True, tables_gen=5)
    e.size(b, {}, c_out=_lib.Outputs())
    assert e.tables.no_net == 1
    assert ("dgen_set_nb_scan", (0,)) in e.lib.calls
    e._tables_gen += 1                     # what set_tariffs / set_switches do
    e.lib.calls.clear()
    e.size(b, {}, c_out=_lib.Outputs())
    assert e.tables.no_net == 0
    assert ("dgen_set_nb_scan", (_lib.NB_CAPM,)) in e.lib.calls
