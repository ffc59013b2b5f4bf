"""numpy restatement of the diffusion step (TEST INFRASTRUCTURE ONLY).

    calc_max_market_share       financial_functions.py:1264-1310
    calc_equiv_time             diffusion_functions_elec.py:343-372
    calc_diffusion_market_share diffusion_functions_elec.py:251-292
    bass_diffusion              diffusion_functions_elec.py:323-338
    calc_diffusion_solar        diffusion_functions_elec.py:24-156 (non-anchor years)

Pinned by tests/golden/diffusion.json (the reference's own functions run on a
synthetic frame, make_golden.py).
"""
import numpy as np


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
