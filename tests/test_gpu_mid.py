"""The mid-size recover kernel (k_recover_mid.hip: 64 signatures per 4-wave workgroup, one role
per wave) against the fixtures, the oracle and the other two recover forms.

Forms are selected with engine knobs (eges_test_set_knob): EGES_LAT_MAX = 0 and EGES_MID_MAX
large send every batch through the mid-size kernel, in its bucket form (EGES_MID_FORM = 2; the
default 1 is auto: bucket while the grid fits one workgroup per CU) or its windowed form (0);
EGES_MID_MAX = 0 sends it through the lane-serial kernel.
Every output byte must agree across forms and with the reference-generated fixtures."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

MID = {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 1 << 20, "EGES_MID_FORM": 2}
MID_WIN = dict(MID, EGES_MID_FORM=0)
MID_B2 = dict(MID, EGES_BKT2=2)  # the bucket form at two workgroups per CU (round 6)
FORMS = {"bucket": MID, "windowed": MID_WIN, "bucket2": MID_B2}
LANE = {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 0}


class knobs:
    def __init__(self, engine, kv):
        self.engine, self.kv = engine, kv

    def __enter__(self):
        self.old = {k: self.engine.get_knob(k) for k in self.kv}
        for k, v in self.kv.items():
            self.engine.set_knob(k, v)

    def __exit__(self, *a):
        for k, v in self.old.items():
            self.engine.set_knob(k, v)


@pytest.mark.parametrize("form", sorted(FORMS))
def test_mid_golden_recover_and_sender(engine, form):
    """every golden recovery item (all reject classes) and every golden sender item through the
    mid-size kernel: byte for byte the fixtures (reference libsecp256k1, oracle/_ref)"""
    MID = FORMS[form]
    g = load_golden("recover.npz")
    with knobs(engine, MID):
        pub, addr, st = engine.ecrecover_batch(g["msg"], g["sig"])
    names = list(g["kind_names"])
    bad = np.nonzero(st != g["status"])[0]
    assert bad.size == 0, [(int(i), names[g["kind"][i]], int(st[i]), int(g["status"][i])) for i in bad[:20]]
    assert np.array_equal(pub, g["pub"])
    with knobs(engine, LANE):
        pub2, addr2, st2 = engine.ecrecover_batch(g["msg"], g["sig"])
    assert np.array_equal(addr, addr2) and np.array_equal(st, st2)
    g2 = load_golden("sender.npz")
    for signer, cid in sorted(set(zip(g2["signer"].tolist(), g2["chain_id"].tolist()))):
        sel = np.nonzero((g2["signer"] == signer) & (g2["chain_id"] == cid))[0]
        with knobs(engine, MID):
            a, s_ = engine.sender_batch(g2["sighash"][sel], g2["r"][sel], g2["s"][sel], g2["v"][sel],
                                        g2["vflags"][sel], int(signer), int(cid))
        assert np.array_equal(s_, g2["status"][sel]), (signer, cid)
        assert np.array_equal(a, g2["addr"][sel]), (signer, cid)


@pytest.mark.parametrize("form", sorted(FORMS))
def test_mid_golden_tiled_ragged(engine, form):
    """the golden recovery set tiled to 10,007 items (ragged last workgroup), device-resident
    entry, mid-size kernel vs the fixtures item for item"""
    import torch
    MID = FORMS[form]
    g = load_golden("recover.npz")
    n = 10007
    rep = -(-n // len(g["msg"]))
    msg = np.tile(g["msg"], (rep, 1))[:n]
    sig = np.tile(g["sig"], (rep, 1))[:n]
    with knobs(engine, MID):
        pub, addr, st = engine.ecrecover_batch_dev(torch.from_numpy(msg).cuda(), torch.from_numpy(sig).cuda(),
                                                   pub=torch.empty((n, 65), dtype=torch.uint8, device="cuda"))
        torch.cuda.synchronize()
    st, pub = st.cpu().numpy(), pub.cpu().numpy()
    assert np.array_equal(st, np.tile(g["status"], rep)[:n])
    assert np.array_equal(pub, np.tile(g["pub"], (rep, 1))[:n])


@pytest.mark.parametrize("form", sorted(FORMS))
@pytest.mark.parametrize("n", [10000, 50000])
def test_mid_adversarial_mix(engine, oracle, n, form):
    """configs[4]'s mix at 10k and 50k through the mid-size kernel: statuses bit-exact against
    their expectation and equal to the lane-serial kernel's, addresses of accepted items the
    signers', a sample of every class against the oracle"""
    import torch
    from eges_amd import txs, workloads
    from eges_amd._lib import SIGNER_EIP155
    msg, sig, exp = engine.synth_sign_dev(300_000 + n, n, 0)
    torch.cuda.synchronize()
    sig_h, msg_h, exp_h = sig.cpu().numpy(), msg.cpu().numpy(), exp.cpu().numpy()
    kind = workloads.adversarial_mix(sig_h, frac=0.10, seed=n)
    r, s, v = workloads.sender_rows_mixed(sig_h, kind, txs.GEEC_CHAIN_ID)
    sig_m = torch.from_numpy(sig_h).cuda()
    rows = [torch.from_numpy(x).cuda() for x in (r, s, v)]
    vf = torch.zeros(n, dtype=torch.uint8, device="cuda")
    out = {}
    for name, kv in (("mid", FORMS[form]), ("lane", LANE)):
        with knobs(engine, kv):
            pub, addr, st = engine.ecrecover_batch_dev(msg, sig_m, pub=torch.empty((n, 65), dtype=torch.uint8,
                                                                                    device="cuda"))
            a2, st2 = engine.sender_batch_dev(msg, *rows, vf, SIGNER_EIP155, txs.GEEC_CHAIN_ID)
            torch.cuda.synchronize()
        out[name] = [x.cpu().numpy() for x in (pub, addr, st, a2, st2)]
    pub, addr, st, a2, st2 = out["mid"]
    for x, y in zip(out["mid"], out["lane"]):
        assert np.array_equal(x, y)
    assert np.array_equal(st, workloads.expected_status(kind, "ecrecover"))
    assert np.array_equal(st2, workloads.expected_status(kind, "sender"))
    assert np.array_equal(addr[st == 0], exp_h[st == 0]) and not addr[st != 0].any()
    assert np.array_equal(a2[st2 == 0], exp_h[st2 == 0]) and not a2[st2 != 0].any()
    for k in range(len(workloads.KIND_NAMES)):
        for i in np.nonzero(kind == k)[0][:6]:
            ost, opub = oracle.recover_pubkey(msg_h[i].tobytes(), sig_h[i].tobytes())
            assert ost == st[i] and (ost != 0 or opub == pub[i].tobytes())


def test_mid_exceptional_joins(engine, oracle):
    """windowed form: the split-form constructions (tests/ecmodel.py) meet the mid-size kernel's
    joins: both the doubling and the infinity branch run, results equal the oracle's; forced redo
    of its loops and comb leaves the golden outputs unchanged"""
    import random

    import ecmodel as M
    MID = MID_WIN
    cases = [c for c in M.recover_cases(random.Random(21), 8) if c[0] in ("split1", "split2")]
    msg = np.frombuffer(b"".join(M.recover_input(c[2], c[3], c[4], c[5])[0] for c in cases), np.uint8).reshape(-1, 32)
    sig = np.frombuffer(b"".join(M.recover_input(c[2], c[3], c[4], c[5])[1] for c in cases), np.uint8).reshape(-1, 65)
    engine.diag_counters(reset=True)
    with knobs(engine, MID):
        pub, addr, st = engine.ecrecover_batch(msg, sig)
    d = engine.diag_counters(reset=True)
    assert d["mid_join"] > 0 and d["mid_redo"] == 0 and d["mid_exc"] == 0, d
    for i in range(len(msg)):
        ost, opub = oracle.recover_pubkey(msg[i].tobytes(), sig[i].tobytes())
        assert ost == st[i] and (ost != 0 or opub == pub[i].tobytes()), i
    assert (st == 6).any() and (st == 0).any()
    g = load_golden("recover.npz")
    with knobs(engine, dict(MID, EGES_TEST_FORCE_REDO=1)):
        pub, addr, st = engine.ecrecover_batch(g["msg"], g["sig"])
    d = engine.diag_counters(reset=True)
    assert np.array_equal(st, g["status"]) and np.array_equal(pub, g["pub"])
    assert d["mid_redo"] > 0, d


def test_bucket_exceptional_joins(engine, oracle):
    """bucket form: u2 values that leave buckets empty (the running sums meet a == b) and u1 chosen
    against u2 R (the final join meets a == +-b, tests/ecmodel.py "join" cases), all through the
    exact branches (mid_join > 0), no bucket addition poisoned (mid_exc == 0), every result the
    oracle's and the lane-serial kernel's; forced redo of the comb keeps the golden outputs"""
    import random

    import ecmodel as M
    from test_exceptional_model import small_u2_cases
    rnd = random.Random(22)
    items = []
    for u2 in small_u2_cases():
        rho, R = M.point_for(rnd.randrange(1, M.N))
        items.append(M.recover_input(rho, R, rnd.randrange(1, M.N), u2))
    for kind, sign, rho, R, u1, u2 in M.recover_cases(rnd, 8):
        if kind == "join":
            items.append(M.recover_input(rho, R, u1, u2))
    msg = np.frombuffer(b"".join(m for m, _ in items), np.uint8).reshape(-1, 32)
    sig = np.frombuffer(b"".join(s_ for _, s_ in items), np.uint8).reshape(-1, 65)
    engine.diag_counters(reset=True)
    with knobs(engine, MID):
        pub, addr, st = engine.ecrecover_batch(msg, sig)
    d = engine.diag_counters(reset=True)
    assert d["mid_join"] > 0 and d["mid_exc"] == 0 and d["mid_redo"] == 0, d
    with knobs(engine, LANE):
        pub2, addr2, st2 = engine.ecrecover_batch(msg, sig)
    assert np.array_equal(pub, pub2) and np.array_equal(st, st2)
    for i in range(len(msg)):
        ost, opub = oracle.recover_pubkey(msg[i].tobytes(), sig[i].tobytes())
        assert ost == st[i] and (ost != 0 or opub == pub[i].tobytes()), i
    assert (st == 6).any() and (st == 0).any()
    g = load_golden("recover.npz")
    with knobs(engine, dict(MID, EGES_TEST_FORCE_REDO=1)):
        pub, addr, st = engine.ecrecover_batch(g["msg"], g["sig"])
    d = engine.diag_counters(reset=True)
    assert np.array_equal(st, g["status"]) and np.array_equal(pub, g["pub"])
    assert d["mid_redo"] > 0 and d["mid_exc"] == 0, d
