#!/usr/bin/env python3
"""Debug helper: a loss-kernel form against form 1 at small shapes (NaN / mismatch census)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import __graft_entry__
    P = __graft_entry__.load_package()
    L = P._lib
    L.load()
    fwd_form, dw_form = int(sys.argv[1]), int(sys.argv[2])
    if len(sys.argv) > 3:
        L.set_tuning("lmloss_splits", int(sys.argv[3]))
    dev = torch.device("cuda:0")
    for (N, H, V) in ((64, 768, 16), (64, 768, 32), (64, 768, 48), (64, 768, 64), (64, 768, 80), (64, 768, 96),
                      (64, 768, 160), (32, 768, 80), (64, 768, 1024)):
        g = torch.Generator(device=dev).manual_seed(0)
        h = torch.randn(N, H, generator=g, device=dev).to(torch.bfloat16)
        w = (0.05 * torch.randn(V, H, generator=g, device=dev)).to(torch.bfloat16)
        y = torch.randint(0, V, (N,), generator=g, device=dev)
        gout = torch.randn(N, generator=g, device=dev)
        res = {}
        for ff, df in ((1, 1), (fwd_form, dw_form)):
            L.set_tuning("lmloss_fwd", ff)
            L.set_tuning("lmloss_dw", df)
            f32 = dict(dtype=torch.float32, device=dev)
            lp, lse, e = torch.empty(N, **f32), torch.empty(N, **f32), torch.empty((N, H), **f32)
            dh = torch.empty((N, H), **f32)
            dw = torch.empty((V, H), **f32)
            ws = torch.empty(L.query("trlx_lmhead_loss_workspace_bytes", N, H, V), dtype=torch.uint8, device=dev)
            s = torch.cuda.current_stream(dev).cuda_stream
            L.call("trlx_lmhead_logprobs_fwd_saved", h.data_ptr(), H, w.data_ptr(), H, N, H, V, y.data_ptr(), 1,
                   lp.data_ptr(), L.F32, lse.data_ptr(), e.data_ptr(), ws.data_ptr(), s)
            L.call("trlx_lmhead_logprobs_bwd", h.data_ptr(), H, w.data_ptr(), H, N, H, V, y.data_ptr(), 1,
                   gout.data_ptr(), L.F32, lse.data_ptr(), e.data_ptr(), dh.data_ptr(), H, L.F32, dw.data_ptr(),
                   L.F32, H, ws.data_ptr(), s)
            torch.cuda.synchronize()
            res[ff] = (lp.cpu(), e.cpu(), dw.cpu())
        a, b = res[1], res[fwd_form]
        bad_lp = (~torch.isclose(a[0], b[0], rtol=1e-4, atol=1e-4)).nonzero().flatten()
        bad_e = (~torch.isclose(a[1], b[1], rtol=1e-2, atol=1e-4)).any(1).nonzero().flatten()
        bad_w = (~torch.isclose(a[2], b[2], rtol=1e-2, atol=1e-5)).any(1).nonzero().flatten()
        print(f"N={N} V={V}: lp bad {len(bad_lp)} first {bad_lp[:8].tolist()} nan {int(b[0].isnan().sum())} | "
              f"E bad rows {len(bad_e)} first {bad_e[:8].tolist()} | dW bad rows {len(bad_w)} first {bad_w[:8].tolist()} "
              f"nan {int(b[2].isnan().any(1).sum())}", flush=True)
    L.set_tuning("lmloss_fwd", 0)
    L.set_tuning("lmloss_dw", 0)


if __name__ == "__main__":
    main()
