"""Run one lm_head variant a few times on one shape (for rocprofv3 PMC passes).
  python tools/lmhead_one.py <variant> <N> <H> <V> [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import __graft_entry__  # noqa: E402

P = __graft_entry__.load_package()


def main():
    var, N, H, V = (int(a) for a in sys.argv[1:5])
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    h = (torch.randn(N, H, generator=g, device=dev) * 0.1).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g, device=dev) * 0.1).to(torch.bfloat16)
    y = torch.randint(0, V, (N,), generator=g, device=dev)
    P._lib.call("trlx_lmhead_set_variant", var)
    for _ in range(reps):
        P.lm_head_logprobs(h, w, y, out_dtype=torch.float32)
    torch.cuda.synchronize()
    print("done", var, N, H, V)


if __name__ == "__main__":
    main()
