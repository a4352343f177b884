"""The RLC root's bucket MSM (rlc_msm.cuh, capi.hip rlc_root_msm_t).  A wrong
root would still give correct verdicts -- the localization tree finds no bad
round and the confirmation passes -- but a clean batch would then build the
trees, so the stages are the observable: on a clean batch the root check
alone must pass.  Both bucket-sum kernels (the load-balanced
k_msm_bucket_seg + k_msm_fixup, default, and one thread per bucket,
DGPU_MSM_SEG=0), G2 and G1 signatures, at a batch size where every list range
holds one entry (buckets cut across many ranges: the fix-up joins the pieces)
and one where ranges hold many entries.  A corrupted batch on each: RLC
reasons equal per-round reasons.  Marked gpu."""
import contextlib

import numpy as np
import pytest

from conftest import open_ctx

pytestmark = pytest.mark.gpu

# ("rlc_bisection" marks every node check's readout, the root's included)
TREE_STAGES = {"rlc_plain_tree", "rlc_leaves_tree", "rlc_confirm"}


@contextlib.contextmanager
def _ctx(seg):
    # the one-thread-per-bucket sums are an A/B variant (the A/B build reads DGPU_MSM_SEG)
    ctx = open_ctx({"DGPU_MSM_SEG": seg, "DGPU_RLC_MIN": "0"} if seg == "0" else {"DGPU_RLC_MIN": "0"})
    try:
        yield ctx
    finally:
        ctx.close()


def _reasons(ctx, code, c, mode, profile=False):
    from drand_amd import _lib
    n = len(c)
    bits = np.zeros((n + 7) // 8, dtype=np.uint8)
    reason = np.zeros(n, dtype=np.uint8)
    pk = np.frombuffer(c.pk, dtype=np.uint8).copy()
    if profile:
        _lib.check(ctx.lib.dgpu_set_profiling(ctx.handle, 1))
    try:
        _lib.check(ctx.lib.dgpu_verify_beacons(ctx.handle, code, _lib.ptr(pk), pk.size, n, _lib.ptr(c.rounds),
                                               _lib.ptr(c.sigs), c.sigs.shape[1], _lib.ptr(c.sig_len),
                                               _lib.ptr(c.prev), c.prev.shape[1], _lib.ptr(c.prev_len), mode, 0x5EED,
                                               _lib.ptr(bits), _lib.ptr(reason)))
        stages = set(_lib.stage_times(ctx)) if profile else set()
    finally:
        if profile:
            _lib.check(ctx.lib.dgpu_set_profiling(ctx.handle, 0))
    return reason, stages


@pytest.mark.parametrize("seg", ["1", "0"])
@pytest.mark.parametrize("code_name,n", [("SCHEME_CHAINED", 3001), ("SCHEME_CHAINED", 180000),
                                         ("SCHEME_UNCHAINED_G1", 3001), ("SCHEME_UNCHAINED_G1", 180000)])
def test_clean_root_passes_and_corrupted_matches_per_round(seg, code_name, n):
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    code = getattr(_lib, code_name)
    if n < 10000:
        # "every list range holds one entry": the MSM_MW = 8 list entries per round
        # (4 MSMs x 2 windows) against the load-balanced kernel's
        # n_cu x 4 SIMDs x 2 waves x 64 threads (capi.hip rlc_root_msm_t)
        import torch
        assert 8 * n <= torch.cuda.get_device_properties(0).multi_processor_count * 512
    c = make_chain(61, n, code, seg_len=64)
    with _ctx(seg) as ctx:
        clean, stages = _reasons(ctx, code, c, _lib.MODE_RLC, profile=True)
        assert not clean.any()
        assert "rlc_root_msm" in stages, " ".join(sorted(stages))
        assert not (stages & TREE_STAGES), " ".join(sorted(stages))
        bad = corrupt(c, 61, rate=3e-4 if n > 10000 else 2e-3)
        rlc, _ = _reasons(ctx, code, c, _lib.MODE_RLC)
        per, _ = _reasons(ctx, code, c, _lib.MODE_PER_ROUND)
    assert sorted(np.nonzero(per)[0].tolist()) == sorted(bad.keys())
    assert rlc.tolist() == per.tolist()
