"""numpy restatement of the diffusion step (TEST INFRASTRUCTURE ONLY).

    calc_max_market_share       financial_functions.py:1264-1310
    calc_equiv_time             diffusion_functions_elec.py:343-372
    calc_diffusion_market_share diffusion_functions_elec.py:251-292
    bass_diffusion              diffusion_functions_elec.py:323-338
    calc_diffusion_solar        diffusion_functions_elec.py:24-156
    anchor-year rescale         diffusion_functions_elec.py:99-133 (anchor())

Pinned by tests/golden/diffusion.json and tests/golden/anchor.json (the
reference's own functions run on synthetic frames, make_golden.py /
make_golden_anchor.py).
"""
import numpy as np

from oracle.market import group_sum_kahan


def max_market_share(payback, sector, curve_sector, curve_pb, curve_mms, all_pb):
    max_pb, min_pb = np.nanmax(all_pb), np.nanmin(all_pb)
    pb = np.asarray(payback, dtype=float).copy()
    pb = np.where(pb >= min_pb, pb, min_pb)
    pb = np.where(pb <= max_pb, pb, max_pb)
    bounded = np.round(pb, 1)
    factor = np.round(bounded * 100)
    table = {}
    for s, p, v in zip(curve_sector, curve_pb, curve_mms):
        table[(s, float(np.round(p * 100)))] = v
    mms = np.array([table.get((s, float(f)), np.nan) for s, f in zip(sector, factor)])
    return bounded, factor, mms


def diffusion(mms, msly, p, q, teq_yr1, dev_w, system_kw, capex, adopt_ly, mv_ly, skc_ly, first):
    mfix = np.where(mms == 0, 1e-9, mms)
    ratio = np.where(msly > mfix, 0, msly / mfix)
    teq = np.log((1 - ratio) / (1 + ratio * (q / p))) / (-1 * (p + q))
    teq2 = teq + teq_yr1 if first else teq + 2
    f = np.e ** (-1 * (p + q) * teq2)
    naf = (1 - f) / (1 + (q / p) * f)
    bms = mms * naf
    dms = np.where(msly > bms, msly, bms)
    ms = np.maximum(dms, msly)
    nms = ms - msly
    nms = np.where(ms > mms, 0, nms)
    na = nms * dev_w
    nmv = na * system_kw * capex
    nskw = na * system_kw
    return dict(mms_fix_zeros=mfix, ratio=ratio, bass_params_teq=teq, teq2=teq2, f=f,
                new_adopt_fraction=naf, bass_market_share=bms, diffusion_market_share=dms,
                market_share=ms, new_market_share=nms, new_adopters=na, new_market_value=nmv,
                new_system_kw=nskw, number_of_adopters=adopt_ly + na, market_value=mv_ly + nmv,
                system_kw_cum=skc_ly + nskw)


def anchor(state, sector, year, dev_w, system_kw_cum, observed):
    """Anchor-year rescale (diffusion_functions_elec.py:99-133): per (state,
    sector, year) group the pandas groupby sum (Kahan, NaN skipped) of the PV
    cumulative capacity and the member count; each agent's share of the group
    total times the observed MW (observed: {(state, sector, year): mw}).
    Returns (system_kw_cum, number_of_adopters, market_share)."""
    kw = np.asarray(system_kw_cum, dtype=float)
    keys = list(zip(state, sector, (int(y) for y in year)))
    groups = {}
    for i, k in enumerate(keys):
        groups.setdefault(k, []).append(i)
    tot = np.empty(len(kw))
    cnt = np.empty(len(kw))
    for k, ix in groups.items():
        tot[ix] = group_sum_kahan(kw[ix])[0]
        cnt[ix] = len(ix)
    with np.errstate(divide="ignore", invalid="ignore"):
        scale = np.where(tot == 0, 1.0 / cnt, kw / tot)
    mw = np.array([observed.get(k, np.nan) for k in keys], dtype=float)
    cum = scale * mw * 1000.0
    adopters = np.where(np.asarray(sector) == "res", cum / 5.0, cum / 100.0)
    w = np.asarray(dev_w, dtype=float)
    with np.errstate(divide="ignore", invalid="ignore"):
        ms = np.where(w == 0, 0.0, adopters / w)
    return cum, adopters, ms
