"""K3 HBM copy sweep: grid size x unroll x nontemporal, interleaved rounds on
one pair of buffers (read + write bytes counted)."""

import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from amdgpu_operator.ops import kernels as K  # noqa: E402


def time_ms(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    out = {}
    for nbytes in (1 << 30, 4 << 30):
        src = torch.empty(nbytes // 4, device="cuda")
        dst = torch.empty_like(src)
        K.fill_uniform_(src, 3)
        arms = {}
        for cus in (128, 256, 512, 1024):
            for variant in range(8):
                arms[f"cus{cus}_v{variant}"] = (lambda c=cus, v=variant: K.hbm_copy(src, dst, c, v))
        arms["torch"] = lambda: dst.copy_(src)
        samples = {k: [] for k in arms}
        for fn in arms.values():
            fn()
        for _ in range(5):
            for k, fn in arms.items():
                samples[k].append(time_ms(fn, 5))
        res = {k: round(2 * nbytes / statistics.median(v) / 1e6, 1) for k, v in samples.items()}
        out[str(nbytes)] = dict(sorted(res.items(), key=lambda kv: -kv[1]))
        del src, dst
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
