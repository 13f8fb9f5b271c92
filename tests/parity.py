"""Parity helpers shared by the GPU tests (oracle vs HIP path)."""
import numpy as np

# north_star: final pose/landmark estimates within 1e-4 relative of the reference path.
EST_RTOL = 1e-4


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


def compare(gpu: dict, ref: dict, rtol=EST_RTOL):
    """Returns a dict of error metrics; asserts nothing."""
    return dict(
        Tcw=row_rel_err(gpu["kf_Tcw"], ref["kf_Tcw"]),
        pt=row_rel_err(gpu["pt_xyz"], ref["pt_xyz"]),
        ln=row_rel_err(gpu["ln_orth"], ref["ln_orth"]),
        chi2_stage=[abs(gpu["chi2"][i] - ref["chi2"][i]) / max(abs(ref["chi2"][i]), 1e-300) for i in range(2)],
        pt_level_diff=int((gpu["ept_level"] != ref["ept_level"]).sum()),
        ln_level_diff=int((gpu["eln_level"] != ref["eln_level"]).sum()),
        pt_bad_diff=int(((gpu["ept_chi2"] > 5.991) | (gpu["ept_depth_ok"] == 0)).astype(int).sum()
                        - ((ref["ept_chi2"] > 5.991) | (ref["ept_depth_ok"] == 0)).astype(int).sum()),
    )
