import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libqattn.so")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def lib():
    import torch  # noqa: F401
    from quantizedattention_amd import _lib
    return _lib.load()


# Bars of the int8 backward's grads against the corrected oracle (relL2 per tensor).  The kernels depart
# from the oracle's rounding in three places (int8_bwd.hip header): fp32 S and P where the reference
# rounds to f16, the RTZ-folded floor of the P quantiser, and bf16 operands for the dV/dK/dQ products.
# The tests print every measured value as "RELL2 int8-bwd-vs-oracle <grad> <value>".  Measured on
# MI355X (round 6, gpurun_out/r06b_rel.log, 114 values): at most 0.0096 on the fixed-shape tests
# (config 3 full length: dk 0.0096, dv 0.0093), at most 0.0344 over the seeded fuzz cases (case 6,
# per-tensor magnitudes up to 16; the next largest 0.0137).  Bars: the measured maximum plus ~1.5x /
# ~1.3x margin (round 5 held every test at 0.05).
INT8_BWD_REL = 0.015
INT8_BWD_REL_FUZZ = 0.045
