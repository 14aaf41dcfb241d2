"""Every batch size at which the default routing changes form (route.hip): the last latency-kernel
batch and the first mid-size one (EGES_LAT_MAX), the last batch of one bucket generation at one
workgroup per CU and the first past it (64 x CUs), the last batch of one generation at two per CU
and the first lane-serial one (128 x CUs). Recovery and VerifySignature, device-resident, with
the default knobs: every address equals the synthetic signer's, every valid signature verifies and
every wrong-key row is rejected, on both sides of each cut (round 6)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sizes(engine):
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    lat = engine.get_knob("EGES_LAT_MAX")
    return sorted({lat, lat + 1, 64 * cus, 64 * cus + 1, 128 * cus, 128 * cus + 1})


def test_routing_cuts_recover_and_verify(engine):
    import torch
    sizes = _sizes(engine)
    top = sizes[-1]
    msg, sig, exp = engine.synth_sign_dev(91 << 24, top, 0)
    pub = torch.empty((top, 65), dtype=torch.uint8, device="cuda")
    engine.ecrecover_batch_dev(msg, sig, pub=pub)
    torch.cuda.synchronize()
    exp_h = exp.cpu().numpy()
    sig64 = sig[:, :64].contiguous()
    publen = torch.full((top,), 65, dtype=torch.uint8, device="cuda")
    wrong = torch.roll(pub, 1, dims=0)
    for n in sizes:
        addr = torch.full((n, 20), 0xEE, dtype=torch.uint8, device="cuda")
        st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        engine.ecrecover_batch_dev(msg[:n], sig[:n], addr=addr, status=st)
        ok = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        engine.verify_batch_dev(pub[:n], publen[:n], msg[:n], sig64[:n], ok=ok)
        bad = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        engine.verify_batch_dev(wrong[:n], publen[:n], msg[:n], sig64[:n], ok=bad)
        torch.cuda.synchronize()
        a, s_ = addr.cpu().numpy(), st.cpu().numpy()
        assert int(s_.max()) == 0 and np.array_equal(a, exp_h[:n]), (n, int((a != exp_h[:n]).any(axis=1).sum()))
        assert int((ok.cpu().numpy() != 1).sum()) == 0, n
        assert int((bad.cpu().numpy() != 0).sum()) == 0, n
