"""Rollout store: one experience chunk pushed and one epoch of training
batches collated, device-resident (PPORolloutStorage: one trlx_rows_copy launch each) vs
the reference path restated (ppo_orchestrator.py:169-187 `.cpu()` x5 + per-sample
PPORLElement lists; ppo_pipeline.py:36-66 pad_sequence collate; accelerate_ppo_model.py:
81-85 `.to(device)`).  Medians of 20.  GPU-box tool:  python tools/store_bench.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import __graft_entry__  # noqa: E402

P = __graft_entry__.load_package()
from oracle import ppo_oracle as orc  # noqa: E402  (the reference collate, restated)


def med(f, reps=20):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    return sorted(ts)[len(ts) // 2]


def main():
    dev = torch.device("cuda:0")
    for name, n, lq, lr, bs in [("C2 chunk 128 x (q 64, r 48), batch 128", 128, 64, 48, 128),
                                ("C4 chunk 128 x (q 128, r 128), batch 32", 128, 128, 128, 32)]:
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randint(1, 32000, (n, lq), generator=g, device=dev)
        r = torch.randint(1, 32000, (n, lr), generator=g, device=dev)
        lp, v, rw = (torch.randn(n, lr, generator=g, device=dev) for _ in range(3))
        nbytes = n * (lq + lr) * 8 + 3 * n * lr * 4

        store = P.PPORolloutStorage(0, dev, capacity=n)

        def dev_push():
            store.clear_history()
            store.push_batch(q, r, lp, v, rw)

        def dev_epoch():
            for b in store.create_loader(bs, shuffle=True):
                pass

        def ref_push():
            qc, rc, lpc, vc, rwc = q.cpu(), r.cpu(), lp.cpu(), v.cpu(), rw.cpu()
            return [P.PPORLElement(qc[i], rc[i], lpc[i], vc[i], rwc[i]) for i in range(n)]

        elems = ref_push()

        def ref_epoch():
            perm = torch.randperm(n)
            for k in range(0, n, bs):
                out = orc.ppo_collate([elems[int(i)] for i in perm[k:k + bs]], 0)
                [t.to(dev) for t in out]

        dev_push()
        t_dp, t_de = med(dev_push), med(dev_epoch)
        t_rp, t_re = med(ref_push), med(ref_epoch)
        print(f"{name}: push {t_dp:8.1f} us device vs {t_rp:8.1f} us reference ({t_rp / t_dp:5.1f}x) | "
              f"epoch of batches {t_de:8.1f} us vs {t_re:8.1f} us ({t_re / t_de:5.1f}x) | chunk bytes {nbytes}",
              flush=True)


if __name__ == "__main__":
    main()
