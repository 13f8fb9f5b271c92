"""Parity helpers shared by the GPU tests (oracle vs HIP path)."""
import json
import os

import numpy as np

# north_star: final pose/landmark estimates within 1e-4 relative of the reference path (reported
# metric, `row_rel_err`). The asserted bar is much tighter: element-wise relative
# 1e-8 where |ref| > 1e-3, absolute 1e-10 elsewhere (observed agreement: 1e-11 .. 1e-15).
EST_RTOL = 1e-4
ELEM_RTOL = 1e-8
ELEM_ATOL = 1e-10
ELEM_BIG = 1e-3


def rel_err(a, b):
    """max |a-b| / max |b| (array-relative, robust to entries near 0)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if b.size == 0:
        return 0.0
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def row_rel_err(a, b):
    """max over rows of |a_i-b_i| / max(|b_i|, 1): per-landmark relative error."""
    if len(b) == 0:
        return 0.0
    a = np.asarray(a, np.float64).reshape(len(a), -1)
    b = np.asarray(b, np.float64).reshape(len(b), -1)
    num = np.abs(a - b).max(axis=1)
    den = np.maximum(np.abs(b).max(axis=1), 1.0)
    return float((num / den).max())


def elem_violation(a, b, rtol=ELEM_RTOL, atol=ELEM_ATOL, big=ELEM_BIG):
    """max over elements of |a-b| / (rtol |b|) where |b| > big, |a-b| / atol elsewhere: <= 1 passes."""
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    if b.size == 0:
        return 0.0
    d = np.abs(a - b)
    scale = np.where(np.abs(b) > big, rtol * np.abs(b), atol)
    return float((d / scale).max())


def assert_parity(m, elem=1.0, north=EST_RTOL):
    """Both bars: the north_star 1e-4 row-relative metric and the element-wise tight bar."""
    log = os.environ.get("PLBA_PARITY_LOG")
    if log:  # diagnostics: every checked metric, one JSON line per check
        with open(log, "a") as f:
            f.write(json.dumps({"test": os.environ.get("PYTEST_CURRENT_TEST", "?"), "elem_bar": elem,
                                **{k: (float(v) if not isinstance(v, list) else [float(x) for x in v])
                                   for k, v in m.items()}}) + "\n")
    assert m["Tcw"] < north and m["pt"] < north and m["ln"] < north, m
    assert m["Tcw_elem"] <= elem and m["pt_elem"] <= elem and m["ln_elem"] <= elem, m


def compare(gpu: dict, ref: dict, rtol=EST_RTOL):
    """Returns a dict of error metrics; asserts nothing."""
    return dict(
        Tcw=row_rel_err(gpu["kf_Tcw"], ref["kf_Tcw"]),
        pt=row_rel_err(gpu["pt_xyz"], ref["pt_xyz"]),
        ln=row_rel_err(gpu["ln_orth"], ref["ln_orth"]),
        Tcw_elem=elem_violation(gpu["kf_Tcw"], ref["kf_Tcw"]),
        pt_elem=elem_violation(gpu["pt_xyz"], ref["pt_xyz"]),
        ln_elem=elem_violation(gpu["ln_orth"], ref["ln_orth"]),
        chi2_stage=[abs(gpu["chi2"][i] - ref["chi2"][i]) / max(abs(ref["chi2"][i]), 1e-300) for i in range(2)],
        pt_level_diff=int((gpu["ept_level"] != ref["ept_level"]).sum()),
        ln_level_diff=int((gpu["eln_level"] != ref["eln_level"]).sum()),
        pt_bad_diff=int(((gpu["ept_chi2"] > 5.991) | (gpu["ept_depth_ok"] == 0)).astype(int).sum()
                        - ((ref["ept_chi2"] > 5.991) | (ref["ept_depth_ok"] == 0)).astype(int).sum()),
    )


def assert_trace_parity(out: dict, ref: dict, rtol=1e-6):
    """The per-iteration trace of BOTH stages: same stage / iteration, the same
    trial count and result while the iteration still makes progress, χ² at linearisation and after
    the trial loop within rtol. (Damped-trial counts are decided by the sign of ρ; once an
    iteration's χ² decrease is at rounding level — converged — that sign is noise on either side.)"""
    tg, tr = out["trace"], ref["trace"]
    assert len(tg) == len(tr) == int(sum(max(i, 0) for i in ref["iters"])), (len(tg), len(tr))
    for i in range(len(tr)):
        for k in ("stage", "iter"):
            assert tg[i][k] == tr[i][k], (i, k, tg[i], tr[i])
        if tr[i]["chi2_start"] - tr[i]["chi2_end"] > 1e-9 * tr[i]["chi2_start"]:
            assert tg[i]["trials"] == tr[i]["trials"] and tg[i]["result"] == tr[i]["result"], (i, tg[i], tr[i])
        for k in ("chi2_start", "chi2_end"):
            assert abs(tg[i][k] - tr[i][k]) <= rtol * abs(tr[i][k]), (i, k, tg[i], tr[i])
