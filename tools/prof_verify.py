"""Small driver for rocprofv3 PMC passes: build a chain on the GPU, run the
per-round verify pipeline `--iters` times (inputs resident in HBM)."""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=131072)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--mode", type=int, default=0)
    a = ap.parse_args()
    import torch
    from drand_amd import _lib
    from drand_amd.chain import get_context
    from drand_amd.synth import make_chain
    torch.cuda.set_device(0)
    c = make_chain(3, a.rounds, _lib.SCHEME_CHAINED, seg_len=max(1, a.rounds // 16384))
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(v).to(dev) for k, v in dict(r=c.rounds.view(np.int64), s=c.sigs, sl=c.sig_len.view(np.int32),
                                                           p=c.prev, pl=c.prev_len.view(np.int32)).items()}
    bits = torch.zeros((a.rounds + 7) // 8, dtype=torch.uint8, device=dev)
    ctx = get_context(0)
    _lib.check(ctx.lib.dgpu_set_pubkey(ctx.handle, _lib.SCHEME_CHAINED, c.pk, 48))
    s = torch.cuda.current_stream(dev)
    for _ in range(a.iters):
        _lib.check(ctx.lib.dgpu_verify_batch_device(ctx.handle, _lib.SCHEME_CHAINED, a.rounds, t["r"].data_ptr(),
                                                    t["s"].data_ptr(), 96, t["sl"].data_ptr(), t["p"].data_ptr(), 96,
                                                    t["pl"].data_ptr(), a.mode, 7, bits.data_ptr(), None,
                                                    ctypes.c_void_p(s.cuda_stream)))
    torch.cuda.synchronize()
    v = np.unpackbits(bits.cpu().numpy(), bitorder="little")[: a.rounds]
    print("valid", int(v.sum()), "of", a.rounds)


if __name__ == "__main__":
    main()
