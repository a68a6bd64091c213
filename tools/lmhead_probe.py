"""Ablation probe of the ping-pong lm_head kernel (variant 5): time with parts of the
pipeline switched off (bit 1: no MFMA, 2: no LDS-DMA staging, 4: no LDS fragment reads).
Results are garbage under ablation; only the times matter.  GPU-box tool."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import __graft_entry__  # noqa: E402

P = __graft_entry__.load_package()
from lmhead_bench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    shapes = [("C4", 16384, 4096, 32128), ("C3", 12288, 768, 32128)]
    for name, N, H, V in shapes:
        g = torch.Generator(device=dev).manual_seed(0)
        h = (torch.randn(N, H, generator=g, device=dev) * 0.1).to(torch.bfloat16)
        w = (torch.randn(V, H, generator=g, device=dev) * 0.1).to(torch.bfloat16)
        y = torch.randint(0, V, (N,), generator=g, device=dev)
        flop = 2.0 * N * H * V
        out = {}
        cfgs = [tuple(int(x) for x in c.split(":")) for c in os.environ.get("PROBE", "8:0,8:8,8:16,5:0").split(",")]
        for rnd in range(3):
            for var, dbg in cfgs:
                P._lib.call("trlx_lmhead_set_variant", var)
                P._lib.set_tuning("lmhead_dbg", dbg)
                t = timeit(lambda: P.lm_head_logprobs(h, w, y, out_dtype=torch.float32))
                out.setdefault(f"v{var}/dbg{dbg}", []).append(t)
        out = {k: (round(sorted(v)[1], 1), round(flop / sorted(v)[1] / 1e6, 1)) for k, v in out.items()}
        P._lib.set_tuning("lmhead_dbg", 0)
        P._lib.call("trlx_lmhead_set_variant", 0)
        print(name, out, flush=True)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
