"""Debug: the per-rank RLC protocol emulated in one process with two contexts."""
import ctypes
import sys
import os
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from drand_amd import _lib
from drand_amd.chain import Verifier
from drand_amd.dist import shard_range
from drand_amd.scheme import get_scheme_by_id_with_default
from drand_amd.synth import corrupt, make_chain

N = 3001
code = _lib.SCHEME_CHAINED
c = make_chain(71, N, code, seg_len=64)
bad = corrupt(c, 71, rate=2e-3)
single = Verifier(get_scheme_by_id_with_default("pedersen-bls-chained")).verify_reasons([c.beacon(i) for i in range(N)], c.pk)
print("bad", sorted(bad.items())[:12])
dev = torch.device("cuda", 0)
ctxs = [_lib.Context(0), _lib.Context(0)]
lib = ctxs[0].lib
rb = lib.dgpu_rlc_root_bytes(code)
roots = torch.zeros(2 * rb, dtype=torch.uint8, device=dev)
pk = np.frombuffer(c.pk, dtype=np.uint8).copy()
keep = []
for world in (1, 2):
    out = []
    for r in range(world):
        lo, hi = shard_range(N, world, r)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a[lo:hi])).to(dev)  # noqa: E731
        d = [t(c.rounds.view(np.int64)), t(c.sigs), t(c.sig_len.view(np.int32)), t(c.prev), t(c.prev_len.view(np.int32))]
        keep.append(d)
        n = hi - lo
        _lib.check(lib.dgpu_rlc_root_device(ctxs[r].handle, code, _lib.ptr(pk), pk.size, n, d[0].data_ptr(),
                                            d[1].data_ptr(), 96, d[2].data_ptr(), d[3].data_ptr(), 96, d[4].data_ptr(),
                                            1000 + 17 * r, roots.data_ptr() + r * rb, None))
    torch.cuda.synchronize()
    for r in range(world):
        lo, hi = shard_range(N, world, r)
        n = hi - lo
        bits = torch.zeros((n + 7) // 8, dtype=torch.uint8, device=dev)
        reason = torch.zeros(n, dtype=torch.uint8, device=dev)
        _lib.check(lib.dgpu_set_profiling(ctxs[r].handle, 1))
        _lib.check(lib.dgpu_rlc_finish_device(ctxs[r].handle, world, roots.data_ptr(), bits.data_ptr(),
                                              reason.data_ptr(), None))
        torch.cuda.synchronize()
        st = _lib.stage_times(ctxs[r])
        _lib.check(lib.dgpu_set_profiling(ctxs[r].handle, 0))
        out.append(reason.cpu().numpy())
        print("world", world, "rank", r, "stages", sorted(st))
    got = np.concatenate(out)
    diff = np.nonzero(got != single)[0]
    print("world", world, "mismatches", len(diff), diff[:10].tolist(), got[diff[:10]].tolist(), single[diff[:10]].tolist())
