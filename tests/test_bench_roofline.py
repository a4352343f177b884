"""bench.py's roofline bookkeeping (host logic only, no GPU): which kernel's
work figure prices each stage, and that every priced stage has one."""
import importlib
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def _bench(monkeypatch, **env):
    for k in ("DGPU_LINES", "DGPU_KB_CHAIN"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    import bench
    return importlib.reload(bench)


def _stages():
    return {"hash_to_g2": 761.0, "h_affine": 9.7, "decode_g2": 107.0, "eng_lines": 697.0, "eng_miller": 1344.0,
            "eng_inv": 14.3, "eng_fe": 509.0, "eng_fe_chain": 782.0, "eng_fe_kbinv": 241.0}


def test_per_thread_stages_priced_by_their_kernels(monkeypatch):
    b = _bench(monkeypatch)
    r = b.roofline_for(_stages(), 10_000_000)
    assert r["kernel"] == "k_eng_miller" and 0.5 < r["frac"] < 1.0
    work = dict(b.hash_work(), **b.engine_work())
    assert b.STAGE_WORK["g2"]["eng_lines"] == "k_lines_thr" and "k_lines_thr" in work
    assert b.KB_STAGE_WORK["eng_fe_chain"] == "k_kb_chain_thr" and "k_kb_chain_thr" in work
    assert set(r["stage_frac"]) == set(_stages()) - {"pack_verdicts"}
    assert all(0.0 < f < 1.0 for f in r["stage_frac"].values())


def test_engine_ab_knobs_switch_the_work_figures(monkeypatch):
    b = _bench(monkeypatch, DGPU_LINES="engine", DGPU_KB_CHAIN="lanes")
    assert b.STAGE_WORK["g2"]["eng_lines"] == "k_eng_lines"
    assert b.KB_STAGE_WORK["eng_fe_chain"] == "k_eng_kb_chain"
    _bench(monkeypatch)


def test_rlc_node_check_stages_not_priced_per_round(monkeypatch):
    """RLC runs the engine stages only for failing tree nodes: they must not be
    priced as if every round ran a pairing."""
    b = _bench(monkeypatch)
    st = {"rlc_hash_to_g2_raw": 300.0, "decode_g2": 360.0, "rlc_leaves_tree": 710.0, "eng_fe": 2.0,
          "eng_fe_chain": 3.0, "eng_fe_kbinv": 1.0, "eng_lines": 1.0, "eng_miller": 2.0}
    r = b.roofline_for(st, 10_000_000, pipeline="rlc")
    assert r["kernel"] == "rlc_leaves_tree"
    assert not any(s.startswith("eng_") for s in r["stage_frac"])


def test_g1_rlc_pipeline_priced(monkeypatch):
    """RLC for G1 signatures prices its own stages (raw G1 hash, G1 decode,
    G1 MSM root, G1 leaves + tree)."""
    b = _bench(monkeypatch)
    st = {"rlc_hash_to_g1_raw": 163.0, "decode_g1": 230.0, "rlc_affine": 5.6, "rlc_root_msm": 38.0,
          "rlc_leaves_tree": 226.0, "eng_miller": 45.0}
    r = b.roofline_for(st, 10_000_000, pipeline="rlc_g1")
    assert r["kernel"] == "k_decode_g1_sigs"
    assert set(r["stage_frac"]) == {"rlc_hash_to_g1_raw", "decode_g1", "rlc_affine", "rlc_root_msm", "rlc_leaves_tree"}
    assert all(0.0 < f < 1.0 for f in r["stage_frac"].values())
