"""Observed parity per GPU test case, printed in pytest's terminal summary (tests/conftest.py).

Every assert_parity call in tests/test_gpu_parity.py records its case, the bound it was held
to and what it measured, so a green run also shows how far inside its bound each case is.
"""
ENTRIES = []


def record(label, variant, max_err, frac_tight, tol):
    ENTRIES.append((label, variant, float(max_err), float(frac_tight), float(tol)))


def lines():
    out = []
    for label, variant, err, frac, tol in ENTRIES:
        out.append(f"{variant:13s} max|gpu-oracle| {err:9.2e}  (bound {tol:7.1e})  frac>5e-5 {frac:8.2e}  {label}")
    return out
