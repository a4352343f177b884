"""The C restatement (oracle/c) against the golden vectors and the Python
oracle (CPU)."""
import hashlib

import numpy as np
import pytest

from conftest import load_golden
from oracle import bls12381 as B


@pytest.fixture(scope="module")
def cref():
    from oracle import c_ref
    c_ref.load()
    return c_ref


def test_hash_to_g2_golden(cref):
    for c in load_golden("hash_to_g2.json")["cases"]:
        assert cref.hash_to_g2(bytes.fromhex(c["msg"])).hex() == c["h"]


def test_hash_to_g2_vs_python(cref):
    for i in range(4):
        m = hashlib.sha256(b"c-vs-py" + bytes([i])).digest()
        assert cref.hash_to_g2(m) == B.g2_compress(B.hash_to_g2(m))


@pytest.mark.parametrize("name", ["chain_chained_s1.json", "chain_unchained_s1.json"])
def test_golden_verdicts_and_reasons(cref, name):
    g = load_golden(name)
    pk = bytes.fromhex(g["pk"])
    chained = g["scheme"] == "pedersen-bls-chained"
    for r in g["rounds"]:
        assert cref.verify_beacon(chained, pk, r["round"], bytes.fromhex(r["prev"]), bytes.fromhex(r["sig"])) == 0
    for c in g["corrupted"]:
        got = cref.verify_beacon(chained, pk, c["round"], bytes.fromhex(c["prev"]), bytes.fromhex(c["sig"]))
        assert got == c["reason"], c["kind"]


def test_batch_threads(cref):
    g = load_golden("chain_chained_s1.json")
    rs = g["rounds"][:8]
    n = len(rs)
    rounds = np.array([r["round"] for r in rs], dtype=np.uint64)
    sigs = np.stack([np.frombuffer(bytes.fromhex(r["sig"]), dtype=np.uint8) for r in rs])
    prev = np.zeros((n, 96), dtype=np.uint8)
    plen = np.zeros(n, dtype=np.uint32)
    for i, r in enumerate(rs):
        p = bytes.fromhex(r["prev"])
        prev[i, : len(p)] = np.frombuffer(p, dtype=np.uint8)
        plen[i] = len(p)
    sigs[3, 0] ^= 0x20
    reason = cref.verify_batch(True, bytes.fromhex(g["pk"]), rounds, sigs, np.full(n, 96, dtype=np.uint32), prev, plen, 4)
    assert reason.tolist() == [0, 0, 0, 3, 0, 0, 0, 0]


def test_hash_to_g1_golden(cref):
    """The C hash to G1 (both DSTs of the G1-signature schemes) == the oracle's fixture."""
    for c in load_golden("hash_to_g1.json")["cases"]:
        if not c["msg"] or "QUUX" in c["dst"]:
            continue
        rfc = "BLS12381G1_XMD" in c["dst"]
        assert cref.hash_to_g1(rfc, bytes.fromhex(c["msg"])).hex() == c["h"]


@pytest.mark.parametrize("name", ["chain_on_g1_s1.json", "chain_g1_rfc9380_s2.json"])
def test_g1_chain_verdicts_and_reasons(cref, name):
    """VerifyBeacon for signatures on G1 in C == the oracle's fixture reasons
    (the C cpu_baseline of configs[3]'s on-G1 chain)."""
    g = load_golden(name)
    rfc = g["scheme"] == "bls-unchained-g1-rfc9380"
    pk = bytes.fromhex(g["pk"])
    for r in g["rounds"][:4]:
        assert cref.verify_beacon_g1(rfc, pk, r["round"], bytes.fromhex(r["sig"])) == 0
    for c in g["corrupted"]:
        assert cref.verify_beacon_g1(rfc, pk, c["round"], bytes.fromhex(c["sig"])) == c["reason"], c["kind"]


def test_recover_golden(cref):
    """Threshold recovery in C (Lagrange in Fr, G2 MSM, VerifyPartial /
    VerifyRecovered pairings) == the oracle's recover fixtures."""
    g = load_golden("recover_t3_n8.json")
    commits = [bytes.fromhex(c) for c in g["commits"]]
    for case in g["cases"]:
        got = cref.recover(commits, g["t"], bytes.fromhex(case["msg"]), [bytes.fromhex(p) for p in case["partials"]])
        assert (got.hex() if got else None) == case["recovered"], case["kind"]


def test_cpu_baseline_reports_host_view():
    """bench.py's cpu_baseline leg on a golden chain: every affinity core as
    threads, `cores` = the measured parallelism (VERDICT r05
    #8), the host / affinity / quota core counts, the
    single-core figure and the all-host-cores projection; verdicts equal the
    fixture's."""
    import numpy as np
    from drand_amd.synth import Chain
    from oracle import cpu_baseline as cb
    g = load_golden("chain_chained_s1.json")
    rows = g["rounds"]
    n = len(rows)
    sigs = np.zeros((n, 96), dtype=np.uint8)
    prev = np.zeros((n, 96), dtype=np.uint8)
    plen = np.zeros(n, dtype=np.uint32)
    for i, r in enumerate(rows):
        s, p = bytes.fromhex(r["sig"]), bytes.fromhex(r["prev"])
        sigs[i, :len(s)] = np.frombuffer(s, dtype=np.uint8)
        prev[i, :len(p)] = np.frombuffer(p, dtype=np.uint8)
        plen[i] = len(p)
    ch = Chain(0, bytes.fromhex(g["pk"]), np.array([r["round"] for r in rows], dtype=np.uint64), sigs,
               np.full(n, 96, dtype=np.uint32), prev, plen, bytes.fromhex(g["genesis"]))
    out = cb.run(ch, 0.2, 2, np.ones(n, dtype=bool))
    assert out["kind"] == "port" and out["sample_verdict_mismatches"] == 0
    assert out["threads"] == 2 and out["host_cores"] >= 1 and out["affinity_cores"] >= 1
    # cores = the measured parallelism (CPU seconds / wall), not the thread count
    assert out["cores"] == round(out["effective_parallelism"], 2) and 0 < out["cores"] <= 2.2
    assert out["projected_all_host_cores_value"] == pytest.approx(out["single_core_value"] * out["host_cores"])
