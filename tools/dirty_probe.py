"""Does a kernel that writes ~0.6 GB (the PPO loss rows' dlogits) slow the NEXT kernel's
reads?  Times the experience forward (2 x 0.6 GB read) after (a) itself, (b) the fused
PPO rows kernel (0.6 GB read + 0.6 GB write), (c) a torch copy of 0.6 GB.  GPU-box tool."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import __graft_entry__  # noqa: E402

P = __graft_entry__.load_package()
from trlx_t5_amd import _lib  # noqa: E402


def main():
    B, T, V = 128, 48, 50257
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    x0 = torch.randn(B, T, V, generator=g, device=dev).to(torch.bfloat16)
    x1 = torch.randn(B, T, V, generator=g, device=dev).to(torch.bfloat16)
    x2 = torch.randn(B, T, V, generator=g, device=dev).to(torch.bfloat16)
    y = torch.randint(0, V, (B, T), generator=g, device=dev)
    lp0, lp1 = torch.empty(B, T, device=dev), torch.empty(B, T, device=dev)
    adv = torch.randn(B, T, device=dev)
    dx = P.grad_buffer_like(x2)
    cp = torch.empty_like(x2)
    s = torch.cuda.current_stream().cuda_stream

    def fwd():
        _lib.call("trlx_lsm_gather_fwd", x0.data_ptr(), x1.data_ptr(), _lib.dtype_code(x0), B, T, V, x0.stride(0),
                  x0.stride(1), y.data_ptr(), y.stride(0), y.stride(1), lp0.data_ptr(), lp1.data_ptr(), _lib.F32,
                  None, None, s)

    def ppo():
        _lib.call("trlx_ppo_policy_fused", x2.data_ptr(), _lib.dtype_code(x2), B, T, V, x2.stride(0), x2.stride(1),
                  y.data_ptr(), y.stride(0), y.stride(1), lp1.data_ptr(), _lib.F32, adv.data_ptr(), None, 1, None,
                  None, float(B * T), 0.2, lp0.data_ptr(), dx.data_ptr(), dx.stride(0), dx.stride(1), s)

    def copy():
        cp.copy_(x2)

    for name, pre in (("after fwd", fwd), ("after ppo rows (R+W)", ppo), ("after torch copy", copy),
                      ("after ppo + 20us idle", None)):
        ts, tp = [], []
        for _ in range(12):
            a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            a.record()
            (pre or ppo)()
            if pre is None:
                torch.cuda._sleep(50000)
            b.record()
            fwd()
            c.record()
            torch.cuda.synchronize()
            ts.append(b.elapsed_time(c) * 1e3)
            tp.append(a.elapsed_time(b) * 1e3)
        ts.sort()
        tp.sort()
        print(f"fwd {name:28s}: median {ts[6]:7.1f} us  ({2 * x0.numel() * 2 / ts[6] / 1e3:6.1f} GB/s); pre {tp[6]:7.1f} us")


if __name__ == "__main__":
    main()
