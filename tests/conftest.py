import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def engine():
    """Initialised engine (GPU tests only)."""
    import eges_amd
    n = eges_amd.init()
    assert n >= 1
    return eges_amd


@pytest.fixture(scope="session")
def oracle():
    from oracle import Oracle
    return Oracle()


# Wire-format sender paths (eges_sender_raw_batch / _dev, eges_block_senders_raw): separate
# tx_rows + prep_sender launches before the recovery (EGES_WIRE_FUSED = 0), and the fused forms,
# where the recovery kernel decodes, hashes and classifies the encodings itself — the mid-size
# kernel's bucket form (k_recover_mid.hip wire_stage / wire_parse) or the latency kernels
# (k_recover_lat.hip, narrow and split), each forced for every batch size with engine knobs.
WIRE_FORMS = {
    "tx_rows": {"EGES_WIRE_FUSED": 0},
    "fused": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 1 << 20, "EGES_MID_FORM": 2, "EGES_WIRE_FUSED": 1},
    "fused_lat": {"EGES_LAT_MAX": 1 << 20, "EGES_WIRE_FUSED": 1},
}


@pytest.fixture(params=sorted(WIRE_FORMS))
def wire_form(request, engine):
    kv = WIRE_FORMS[request.param]
    old = {k: engine.get_knob(k) for k in kv}
    for k, v in kv.items():
        engine.set_knob(k, v)
    yield request.param
    for k, v in old.items():
        engine.set_knob(k, v)


def load_golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
