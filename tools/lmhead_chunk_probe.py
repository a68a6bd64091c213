"""Probe for the §8f-2 long-K route: can hipBLASLt GEMMs over vocab chunks, each chunk's
row reductions running on a second stream while the next chunk's GEMM computes, beat
"full GEMM (writes all [N, V] logits) + rows"?  The ring of chunk buffers is small enough
to sit in the 256 MB Infinity Cache.  Row work is proxied by the experience rows kernel on
the chunk (same bytes / VALU per element as a partial (max, Σexp) pass).

GPU-box tool:  python tools/lmhead_chunk_probe.py  (HIP events, medians of interleaved rounds)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import __graft_entry__  # noqa: E402

P = __graft_entry__.load_package()


def timeit(fn, reps=7):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    dev = torch.device("cuda:0")
    print("blas:", torch.backends.cuda.preferred_blas_library(), flush=True)
    N, H, V = int(os.environ.get("N", 16384)), int(os.environ.get("H", 4096)), int(os.environ.get("V", 32128))
    g = torch.Generator(device=dev).manual_seed(0)
    h = (torch.randn(N, H, generator=g, device=dev) * 0.1).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g, device=dev) * 0.1).to(torch.bfloat16)
    y = torch.randint(0, V, (N,), generator=g, device=dev)
    logits = torch.empty(N, V, dtype=torch.bfloat16, device=dev)
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)

    def full():
        torch.matmul(h, w.t(), out=logits)
        P.logprobs_from_logits(logits, y)

    def gemm_only():
        torch.matmul(h, w.t(), out=logits)

    def chunked(vc, depth, overlap):
        nch = (V + vc - 1) // vc
        ring = [torch.empty(N * vc, dtype=torch.bfloat16, device=dev) for _ in range(depth)]
        yc = [(y - c * vc).clamp_(0, min(vc, V - c * vc) - 1) for c in range(nch)]
        ev_g = [torch.cuda.Event() for _ in range(nch)]
        ev_r = [torch.cuda.Event() for _ in range(nch)]

        def run():
            for c in range(nch):
                v0, v1 = c * vc, min(V, (c + 1) * vc)
                buf = ring[c % depth][:N * (v1 - v0)].view(N, v1 - v0)
                if overlap and c >= depth:
                    main_s.wait_event(ev_r[c - depth])
                torch.matmul(h, w[v0:v1].t(), out=buf)
                if overlap:
                    ev_g[c].record(main_s)
                    side.wait_event(ev_g[c])
                    with torch.cuda.stream(side):
                        P.logprobs_from_logits(buf, yc[c])
                    ev_r[c].record(side)
                else:
                    P.logprobs_from_logits(buf, yc[c])
            if overlap:
                main_s.wait_stream(side)
        return run

    def token_chunked(nc):
        ring = torch.empty(nc * V, dtype=torch.bfloat16, device=dev)

        def run():
            for n0 in range(0, N, nc):
                n1 = min(N, n0 + nc)
                buf = ring[:(n1 - n0) * V].view(n1 - n0, V)
                torch.matmul(h[n0:n1], w.t(), out=buf)
                P.logprobs_from_logits(buf, y[n0:n1])
        return run

    cases = {"full gemm+rows": full, "full gemm only": gemm_only}
    if os.environ.get("VCHUNKS", "0") == "1":
        for vc in (2048, 4096, 8192):
            for depth in (2, 3):
                cases[f"chunk {vc} depth {depth} overlap"] = chunked(vc, depth, True)
            cases[f"chunk {vc} serial"] = chunked(vc, 2, False)
    for nc in (1024, 2048, 4096, 8192):
        cases[f"token chunk {nc} serial"] = token_chunked(nc)
    res = {}
    for rnd in range(3):
        for k, fn in cases.items():
            res.setdefault(k, []).append(timeit(fn))
        print(f"round {rnd} done", flush=True)
    base = sorted(res["full gemm+rows"])[1]
    for k, v in res.items():
        m = sorted(v)[1]
        print(f"{k:34s} {m:9.1f} us  {2.0 * N * H * V / m / 1e6:7.1f} TFLOP/s  vs full gemm+rows {base / m:5.3f}x",
              flush=True)


if __name__ == "__main__":
    main()
