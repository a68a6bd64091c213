#!/usr/bin/env python3
"""bench.py — PPO experience+loss hot path throughput on MI355X.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5] [--cpu-seconds S]

One "step" = one PPOHotPath.step over one shard of synthetic rollouts (see
trlx-t5_amd/step.py): policy+reference log-softmax-gather (experience), fused KL reward
+ GAE + whitening moments (+ RCCL all-reduce when N > 1), fused new-policy logprob + PPO
gradient + dlogits write, value loss + stats; the score RunningMoments / clip and the
adaptive KL controller run on device inside the two rollout tails (PPOControlState,
configs/ppo_config.yml settings; --host-state for a host-constant beta).  Inputs are resident in HBM before timing.
Weak scaling: every rank processes its own shard of the configuration's per-GPU batch;
`value` = all ranks' tokens / max-over-ranks wall time.

--config c5 times the ILQL loss instead (ILQLHotPath.step: prep, rows, finalize launches;
tokens = action tokens; no collective — the reference's ILQL loss is rank-local).

Prints ONE JSON line on rank 0 (contract in the task statement), with
  roofline      dominant kernel's algorithmic bytes / its average HIP-event time vs 8 TB/s
  cpu_baseline  the oracle (op-for-op reference PyTorch path) on host cores, bounded sample
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "PPO experience+loss tokens/sec and % HBM roofline, 1/2/4/8 MI355X"
METRIC_ILQL = "ILQL loss (fwd+bwd) action tokens/sec and % HBM roofline, MI355X (config 5, not the headline)"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip-level table)
TIMER_EVERY = 4        # instrument one step in four: HIP events around the vocab-row launches (>= 5 samples
                       # in a 20-step run; a fully instrumented C2 step costs ~1.7 %, so one in four ~0.4 %)
SETTLE_MAX_STEPS = 5000
C3_GLOBAL_BATCH = 512  # BASELINE.json configs[2]: "batch 512, DP over 2/4 GPUs"

CONFIGS = {
    # name: (rows per GPU, response tokens, vocab, description)      BASELINE.json configs[]
    "c2": (128, 48, 50257, "C2 GPT-2 sentiments PPO shape: 128 x 48 response tokens, vocab 50257, bf16 logits"),
    "c3": (256, 48, 32128, "C3 T5-base seq2seq PPO: 256 rows/GPU x 48 decoder tokens (decoder-length masked), vocab 32128"),
    "c4": (128, 128, 32128, "C4 UL2-20B rl_ul2 shape: 128 rows/GPU x 128 decoder tokens, vocab 32128, bf16 logits"),
    "c5": (128, 64, 50257, "C5 ILQL sentiments loss: 128 rows/GPU x 64 tokens (63 actions), vocab 50257, fp32 "
                           "logits + 2 Q + 2 target-Q heads"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    p.add_argument("--cpu-seconds", type=float, default=8.0,
                   help="CPU baseline budget per logits dtype (0 = skip); PPO times bf16 and fp32")
    p.add_argument("--settle-ms", type=float, default=200.0,
                   help="after the W warm-up steps keep stepping until the GPU has been busy this long: an "
                        "idle MI355X runs this step up to ~20%% slow for its first ~20-40 ms of load "
                        "(profiles/r02_slowstart.log); reported as warmup_steps_run / warmup_ms (0 = off)")
    p.add_argument("--no-fp32-line", action="store_true",
                   help="PPO C2 at N=1: skip the secondary fp32-logits measurement (reported under fp32_logits)")
    p.add_argument("--no-timers", action="store_true", help="skip per-kernel HIP events")
    p.add_argument("--no-from-hidden", action="store_true",
                   help="PPO C2 at N=1: skip the secondary §8f-2 loss-side measurement (reported under from_hidden: "
                        "the PPO update from hidden states, fused MFMA route vs the hipBLASLt logits route)")
    p.add_argument("--from-hidden-steps", type=int, default=10,
                   help="updates per route and round of the from_hidden measurement (3 interleaved rounds)")
    p.add_argument("--host-state", action="store_true",
                   help="PPO: keep beta as a host constant and skip the score RunningMoments/clip and the KL "
                        "controller update (the default runs them on device, ppo_config.yml settings)")
    p.add_argument("--logits-dtype", default="bf16", choices=("bf16", "fp32"),
                   help="PPO logits dtype (bf16: the T5/UL2 path and BASELINE's C2 row; fp32: the reference's GPT "
                        "path)")
    p.add_argument("--overlap-tail", action="store_true",
                   help="PPO: run the loss tail on a side stream beside the next step's experience rows (measured "
                        "~1 %% slower than the default in-stream tail: the cross-stream event waits cost more than "
                        "the ~9 us tail, profiles/r02_schedules.log)")
    p.add_argument("--tune", action="append", default=[],
                   help="key=value launch tuning (trlx_set_tuning; A/B only, results identical)")
    p.add_argument("--global-batch", type=int, default=0,
                   help="strong scaling: fix the GLOBAL rollout count (rows per GPU = G / N; SURVEY §8d runs C4 "
                        "at 1024 rows on 1/2/4/8 GPUs); default 0 = the config's rows per GPU (weak scaling)")
    p.add_argument("--loss-norm", default="rank", choices=("rank", "global"),
                   help="PPO loss normalisers for N > 1: rank-local Σmask (the reference) or the global Σmask "
                        "(carried by the whitening all-reduce)")
    p.add_argument("--no-defer-tail", action="store_true",
                   help="PPO serial schedule: run each loss tail as its own launch (default: folded into the next "
                        "step's experience rows launch, PPOHotPath(defer_tail=True); the last one is flushed inside "
                        "the timed region)")
    p.add_argument("--split-beta", action="store_true",
                   help="A/B: the serial schedule with the split-beta kernels the pipelined schedule runs")
    p.add_argument("--coef-launch", action="store_true",
                   help="A/B: split-beta loss rows read coefficients from their own launch instead of deriving them")
    p.add_argument("--no-gae-fold", action="store_true",
                   help="A/B: pipelined schedule with GAE(k+1) as its own launch instead of the first workgroups of "
                        "the L rows(k) launch")
    p.add_argument("--schedule", default="auto", choices=("auto", "serial", "pipelined"),
                   help="PPO: serial = PPOHotPath.step per batch (three launches: E rows, GAE, L rows); pipelined = "
                        "pipeline_step (two launches per batch: the next batch's GAE rides the loss rows launch, "
                        "and the next batch's experience rows run while this batch's whitening all-reduce is in "
                        "flight; results bit-identical to step(split_beta=True)); auto = pipelined")
    p.add_argument("--dist", action="store_true",
                   help="initialise the process group even at world size 1 (rehearses the RCCL path on one GPU: "
                        "the whitening all-reduce then runs through RCCL every step)")
    p.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                   help="process-group backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse "
                        "several ranks on one GPU)")
    p.add_argument("--comm", default="auto", choices=("auto", "rccl", "torch"),
                   help="collectives of the PPO step under a process group: rccl = the boundary's RCCL helper "
                        "(comm.RcclComm: ncclAllReduce enqueued on the step's stream, no ProcessGroupNCCL event "
                        "joins); torch = torch.distributed.all_reduce; auto = rccl with the nccl backend, falling "
                        "back to torch (reported in config.comm) if the communicator cannot be created")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher rehearsal without a GPU: every rank joins a gloo group, checks its rank / world "
                        "against the others and rank 0 prints one JSON line (tests/test_host_cpu.py)")
    p.add_argument("--rank-timeout", type=float, default=600.0,
                   help="--gpus N launcher deadline in seconds: ranks still running then are stopped (SIGTERM, "
                        "then SIGKILL), named on stderr, and the launcher exits 124 (0 = no deadline)")
    p.add_argument("--dry-run-hang-rank", type=int, default=-1, help=argparse.SUPPRESS)  # launcher test: a stuck rank
    return p.parse_args()


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


RANK_KILL_GRACE_S = 10.0  # after SIGTERM, how long a rank gets before SIGKILL
RC_RANK_TIMEOUT = 124     # launcher exit code when the deadline fired (as timeout(1))


def _stop_ranks(procs, live, why):
    """SIGTERM every live rank, SIGKILL the ones still alive after the grace period; by PID
    (never by pattern).  Returns the ranks that had to be killed."""
    import signal
    for q in live:
        q.send_signal(signal.SIGTERM)
    t_end = time.monotonic() + RANK_KILL_GRACE_S
    while any(q.poll() is None for q in live) and time.monotonic() < t_end:
        time.sleep(0.05)
    killed = [procs.index(q) for q in live if q.poll() is None]
    for q in live:
        if q.poll() is None:
            q.send_signal(signal.SIGKILL)
    if killed:
        print(f"bench.py launcher: ranks {killed} ignored SIGTERM ({why}); killed", file=sys.stderr)
    return killed


def launch_ranks(n, argv, timeout_s=600.0):
    """`bench.py --gpus N` without an external launcher: start N child processes of this
    script (one per GPU, RANK = LOCAL_RANK = i, WORLD_SIZE = N, rendezvous on 127.0.0.1) and
    return the first non-zero exit code.  Runs BEFORE anything in this process touches the
    GPU (torch is not even imported) and never execs: the parent only waits.  Rank 0's
    stdout carries the JSON line; if a rank fails, the others are terminated by PID.
    Deadline (--rank-timeout): a rank that neither finishes nor fails — e.g. one blocked in
    ncclCommInitRank after a peer died — would otherwise hold the parent until the driver's
    own limit; when `timeout_s` expires every live rank gets SIGTERM, then SIGKILL, the
    ranks that had not exited are named on stderr and the launcher returns 124."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    live = list(procs)
    deadline = time.monotonic() + timeout_s if timeout_s and timeout_s > 0 else None
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"bench.py launcher: rank {procs.index(p)} exited with {code}; stopping the others",
                      file=sys.stderr)
                _stop_ranks(procs, live, f"rank {procs.index(p)} failed")
        if live and deadline is not None and time.monotonic() >= deadline:
            stuck = [procs.index(q) for q in live]
            print(f"bench.py launcher: --rank-timeout {timeout_s:g} s expired; ranks {stuck} had not exited; "
                  f"stopping them", file=sys.stderr)
            _stop_ranks(procs, live, "deadline")
            rc = rc or RC_RANK_TIMEOUT
            break
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


def resolve_shape(args, world):
    """(rows per GPU, T, V, workload description) of this run; sets args.global_batch when
    the config fixes the global batch.  C3 at N > 1 defaults to BASELINE.json's global batch of
    512 (T5-base, "batch 512, DP over 2/4 GPUs": strong scaling, 256 / 128 rows per GPU); at
    N = 1 it runs one 256-rollout DP2 shard.  Every other config defaults to its rows per GPU
    (weak scaling) unless --global-batch is given."""
    B, T, V, desc = CONFIGS[args.config]
    if args.config == "c3" and world > 1 and not args.global_batch:
        args.global_batch = C3_GLOBAL_BATCH
        desc = f"{desc} (BASELINE C3 global batch {C3_GLOBAL_BATCH})"
    if args.global_batch:
        if args.global_batch % world:
            raise SystemExit(f"--global-batch {args.global_batch} is not divisible by {world} ranks")
        B = args.global_batch // world
        desc = f"{desc}; strong scaling: {args.global_batch} rollouts global, {B} per GPU"
    return B, T, V, desc


def dry_run(args):
    """Rehearse the rank layout of a multi-rank run on the CPU (gloo): each rank contributes
    its RANK / LOCAL_RANK and rank 0 checks the group saw 0..N-1 exactly once."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if rank == args.dry_run_hang_rank:  # a rank that never finishes (and ignores SIGTERM)
        import signal
        signal.signal(signal.SIGTERM, signal.SIG_IGN)
        while True:
            time.sleep(1)
    B, T, V, desc = resolve_shape(args, world)
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))  # a stand-in for the timed region: per-rank clocks differ
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        got = [None] * world
        dist.all_gather_object(got, (rank, local, elapsed))
        dist.destroy_process_group()
    else:
        got = [(rank, local, elapsed)]
    if rank == 0:
        per_rank = [g[2] for g in sorted(got)]
        got = [g[:2] for g in got]
        ok = sorted(got) == [(r, r) for r in range(world)]
        print(json.dumps({"dry_run": True, "n_gpus": world, "requested": args.gpus, "ranks": got, "ok": ok,
                          "config": {"workload": desc, "rows_per_gpu": B, "global_batch": B * world,
                                     "scaling": "strong" if args.global_batch else "weak",
                                     "comm_nranks": world},
                          "rank_ms_per_step": {"min": round(min(per_rank) * 1e3, 4),
                                               "max": round(max(per_rank) * 1e3, 4), "ranks": len(per_rank)}}),
              flush=True)
        if not ok:
            raise SystemExit(3)


def algorithmic_bytes(V, s, masked, pipelined=False, fill=1.0):
    """Minimum HBM bytes per response token, per launch.  Each [B,T] fp32
    vector read or written once counts 4 B; int64 labels / mask 8 B.  pipelined: the
    split-beta kernels (GAE -> A0, Ak, kl, score terms; the loss rows finish rewards and
    returns), the GAE riding the loss rows launch.  fill (a ragged batch, C3): the fraction
    of decoder positions inside their rollout's length — only those logits rows are read
    (experience: store padding past the length; loss: mask == 0), while every dlogits row is
    written (zeros where masked)."""
    mask_b = 8 if masked else 0
    exp = 2 * V * s * fill + 8 + 2 * 4             # K1 rows: policy + ref row, label -> lp, ref_lp
    row = V * s * fill + V * s                      # loss row read + dlogits row written
    if pipelined:
        gae = 3 * 4 + 4 * 4 + mask_b               # lp, ref_lp, values -> adv0, adv_kl, rew_kl, rew_score
        loss = row + 8 + 4 * 7 + 4 * 4 + mask_b + gae  # row + dlogits, label, 7 vectors -> lp, dv, rewards, returns
    else:
        gae = 2 * 4 + 4 + 3 * 4 + mask_b           # lp, ref_lp, values -> rewards, adv, returns
        loss = row + 8 + 4 * 6 + 2 * 4 + mask_b    # K2 rows: row + dlogits, label, 6 vectors -> lp, dv
    lred = 11 * 4                                  # per-token loss record read back
    return {"experience": exp, "loss": loss, "step": exp + gae + loss + lred - (gae if pipelined else 0)}


def ilql_algorithmic_bytes(B, L, V, s, nq=2):
    """Minimum HBM bytes of one ILQL rows launch: every logits row but the last and every
    Q row read once, every gradient row written once (the last logits row's gradient is
    zeros, write-only); target-Q rows cost two 4-B gathers per action; small [B, .] tensors
    (ids, masks, rewards, vs, dvs, records) read / written once."""
    A = L - 1
    rows = (B * (L - 1) + nq * B * A) * V * s + (B * L + nq * B * A) * V * s
    small = B * A * (nq * s + 8 + 8 + 4 + 4 + 4 + 16 * (1 + nq)) + B * L * (8 + 8)
    return rows + small


def make_ilql_inputs(torch, P, B, L, V, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    A = L - 1
    f = dict(generator=g, device=dev)
    logits = torch.randn(B, L, V, **f)
    qs = [torch.randn(B, A, V, **f) for _ in range(2)]
    tqs = [q + 0.1 * torch.randn(B, A, V, **f) for q in qs]
    vs = torch.randn(B, L, **f)
    ids = torch.randint(0, V, (B, L), **f)
    dones = torch.ones(B, L, dtype=torch.long, device=dev)
    dones[:, -1] = 0
    batch = P.ILQLBatch(ids, torch.ones(B, L, dtype=torch.long, device=dev), torch.randn(B, A, **f),
                        torch.arange(L, device=dev).repeat(B, 1), torch.arange(A, device=dev).repeat(B, 1), dones)
    torch.cuda.synchronize()
    return logits, qs, tqs, vs, batch


def ilql_cpu_baseline(torch, L, V, seconds):
    """Oracle ILQL loss (reference ops, fp32, autograd backward) on host cores."""
    from oracle import ppo_oracle as orc
    cores = _cores()
    torch.set_num_threads(cores)
    Bs, A = 2, L - 1
    g = torch.Generator().manual_seed(123)
    logits = torch.randn(Bs, L, V, generator=g)
    qs = [torch.randn(Bs, A, V, generator=g) for _ in range(2)]
    tqs = [torch.randn(Bs, A, V, generator=g) for _ in range(2)]
    vs = torch.randn(Bs, L, 1, generator=g)
    ids = torch.randint(0, V, (Bs, L), generator=g)
    dones = torch.ones(Bs, L, dtype=torch.long)
    dones[:, -1] = 0
    rew = torch.randn(Bs, A, generator=g)
    toks, t0 = 0, time.perf_counter()
    while True:
        lg = logits.clone().requires_grad_(True)
        q = [x.clone().requires_grad_(True) for x in qs]
        v = vs.clone().requires_grad_(True)
        loss, _ = orc.ilql_loss(lg, q, tqs, v, ids, torch.ones(Bs, L, dtype=torch.long), rew,
                                torch.arange(A).repeat(Bs, 1), dones)
        loss.backward()
        toks += Bs * A
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": toks / el, "unit": "tokens/s", "cores": cores, "affinity_cores": affinity_cores(), "kind": "port",
            "sample": f"{toks // (Bs * A)} steps of {Bs}x{L}x{V} fp32 (oracle.ilql_loss: reference ops incl. "
                      f"autograd backward), {el:.1f} s, torch.set_num_threads({cores})"}


def affinity_cores():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _cores():
    """Threads the CPU baseline uses: every core in this process's affinity mask, unless the
    environment caps the process's share (OMP_NUM_THREADS: the GPU box sets it to its 16-core
    share per GPU while sched_getaffinity shows the whole machine)."""
    cores = affinity_cores()
    cap = os.environ.get("OMP_NUM_THREADS", "")
    if cap.isdigit() and int(cap) > 0:
        cores = min(cores, int(cap))
    return max(1, cores)


def make_inputs(torch, B, T, V, dev, seed, masked, dtype=None):
    g = torch.Generator(device=dev).manual_seed(seed)
    bf = dtype or torch.bfloat16
    logits = torch.randn(B, T, V, generator=g, device=dev, dtype=torch.float32).to(bf)
    ref_logits = (logits.float() + 0.1 * torch.randn(B, T, V, generator=g, device=dev)).to(bf)
    new_logits = (logits.float() + 0.05 * torch.randn(B, T, V, generator=g, device=dev)).to(bf)
    labels = torch.randint(0, V, (B, T), generator=g, device=dev)
    old_values = torch.randn(B, T, generator=g, device=dev)
    values = old_values + 0.3 * torch.randn(B, T, generator=g, device=dev)
    scores = torch.rand(B, generator=g, device=dev) * 24 - 12
    lengths = mask = None
    if masked:  # decoder lengths L ~ U{1..T}, zero right-padding (ppo_pipeline.py:47-65)
        lengths = torch.randint(1, T + 1, (B,), generator=g, device=dev)
        mask = (torch.arange(T, device=dev)[None, :] < lengths[:, None]).long()
        old_values = old_values.masked_fill(mask == 0, 0)
    torch.cuda.synchronize()
    return dict(logits=logits, ref_logits=ref_logits, new_logits=new_logits, labels=labels,
                old_values=old_values, values=values, scores=scores, lengths=lengths, mask=mask)


def cpu_baseline(torch, T, V, seconds, dtype=None):
    """Oracle (reference PyTorch ops, in the logits dtype: native bf16 like the T5/UL2 path, or
    fp32 like the GPT path) on host cores."""
    from oracle import ppo_oracle as orc
    cores = _cores()
    torch.set_num_threads(cores)
    Bs = 8
    g = torch.Generator().manual_seed(123)
    bf = dtype or torch.bfloat16
    logits = torch.randn(Bs, T, V, generator=g).to(bf)
    ref_logits = (logits.float() + 0.1 * torch.randn(Bs, T, V, generator=g)).to(bf)
    new_logits = (logits.float() + 0.05 * torch.randn(Bs, T, V, generator=g)).to(bf)
    labels = torch.randint(0, V, (Bs, T), generator=g)
    old_values = torch.randn(Bs, T, generator=g).to(bf)
    values = (old_values.float() + 0.3 * torch.randn(Bs, T, generator=g)).to(bf)
    scores = torch.rand(Bs, generator=g) * 24 - 12
    sc = orc.ScoreControl(False, 10)
    kl = orc.AdaptiveKLController(0.05, 6, 10000)
    toks, t0 = 0, time.perf_counter()
    while True:
        s_t, _, _ = sc(scores)
        r = orc.ppo_step_reference(logits, ref_logits, new_logits, labels, old_values, values, s_t,
                                   kl_coef=kl.value)
        kl.update(float(r["stats"]["policy/approx_kl"]), n_steps=Bs)
        toks += Bs * T
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": toks / el, "unit": "tokens/s", "cores": cores, "affinity_cores": affinity_cores(), "kind": "port",
            "sample": f"{toks // (Bs * T)} steps of {Bs}x{T}x{V} {str(bf).replace('torch.', '')} (oracle ScoreControl + ppo_step_reference + "
                      f"AdaptiveKLController: reference ops incl. autograd backward), {el:.1f} s, torch.set_num_threads({cores})"}


MFMA_BF16_PEAK_TFLOPS = 2516.6  # dense bf16: 1024 FLOP/clk/SIMD x 4 SIMD x 256 CU x 2.4 GHz (MI355X_MICROARCH.md)
FROM_HIDDEN_SHAPES = {  # name: (rows, T, V, H, masked) — BASELINE configs[1] and a configs[2] DP2 shard
    "c2": (128, 48, 50257, 768, False),
    "c3_shard": (256, 48, 32128, 768, True),
}


def from_hidden_leg(torch, P, dev, name, steps, rounds=3):
    """§8f-2, loss side, as the driver runs it: the PPO update from the policy's hidden states
    after one experience_from_hidden, `steps` updates per route per round, rounds interleaved
    (the first route rotates), HIP events on the launch stream around each round; the deferred
    loss tail of every hot-path update runs inside the timed region.  Per-update times are the
    median over rounds.  Routes:
      fused         PPOHotPath.policy_loss_from_hidden (csrc/lmhead_loss.hip: no [N, V] logits /
                    dlogits in HBM; tokens with mask == 0 compacted out of the MFMA passes)
      gemm          the reference's structure on the hot path's kernels: hipBLASLt bf16 logits ->
                    fused loss rows -> hipBLASLt dh and dW GEMMs, over every token of the padded
                    batch (the reference computes masked logits: accelerate_ppo_model.py:96-111)
      gemm_compact  (masked shapes) the same kernels over the live tokens only: the live hidden
                    rows (and their per-token inputs) gathered, the gemm route on a [1, live]
                    batch, dh scattered back — the kernel-for-kernel comparison with `fused`
                    (the live-row index is built once per batch outside the timed region:
                    torch.nonzero syncs the host; the gathers and the scatter are timed)
      dropin        the drop-in surface a reference user calls: PPOConfig.loss_from_hidden
                    (autograd through lm_head_logprobs — saved-P plan — and the PPO loss) +
                    loss.backward(), grads set to None each update (zero_grad(set_to_none)); no
                    compaction (the reference's mask enters the loss only)"""
    B, T, V, H, masked = FROM_HIDDEN_SHAPES[name]
    g = torch.Generator(device=dev).manual_seed(4242)
    f = dict(generator=g, device=dev)
    h = torch.randn(B, T, H, **f).to(torch.bfloat16)
    w = (0.05 * torch.randn(V, H, **f)).to(torch.bfloat16)
    ref_h = (h.float() + 0.1 * torch.randn(B, T, H, **f)).to(torch.bfloat16)
    new_h = (h.float() + 0.05 * torch.randn(B, T, H, **f)).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, T), **f)
    old_values = torch.randn(B, T, **f)
    values = old_values + 0.3 * torch.randn(B, T, **f)
    scores = torch.rand(B, **f) * 24 - 12
    lengths = mask = None
    if masked:
        lengths = torch.randint(1, T + 1, (B,), **f)
        mask = (torch.arange(T, device=dev)[None, :] < lengths[:, None]).long()
    cfg = P.PPOConfig()
    hp = P.PPOHotPath(cfg, B, T, V, torch.bfloat16, dev, kl_coef=0.05, defer_tail=True)
    hp.experience_from_hidden(h, w, ref_h, w, labels, old_values, scores, lengths=lengths, mask=mask, route="fused")
    hp.wait_stats()
    routes = {"fused": lambda: hp.policy_loss_from_hidden(new_h, w, labels, values, old_values, mask=mask,
                                                          route="fused"),
              "gemm": lambda: hp.policy_loss_from_hidden(new_h, w, labels, values, old_values, mask=mask,
                                                         route="gemm")}
    nv = int(mask.sum().item()) if masked else B * T
    hpc = None
    if masked:  # gemm over the live tokens: a [1, nv] hot path fed the gathered rows
        idx = mask.reshape(-1).nonzero().squeeze(1)
        hpc = P.PPOHotPath(cfg, 1, nv, V, torch.bfloat16, dev, kl_coef=0.05, defer_tail=True)
        hpc.adv_stats.copy_(hp.adv_stats)  # the batch's whitening record (Σmask = nv at [3])
        dh_full = torch.zeros(B * T, H, dtype=torch.bfloat16, device=dev)

        def gemm_compact():
            hc = new_h.reshape(B * T, H).index_select(0, idx).view(1, nv, H)
            for dst, src in ((hpc.lp_old, hp.lp_old), (hpc.adv_raw, hp.adv_raw), (hpc.returns, hp.returns)):
                torch.index_select(src.reshape(-1), 0, idx, out=dst.view(-1))
            take = lambda t: t.reshape(-1).index_select(0, idx).view(1, nv)  # noqa: E731
            _, _, dhc, _, _ = hpc.policy_loss_from_hidden(hc, w, take(labels), take(values), take(old_values),
                                                          route="gemm")
            dh_full.index_copy_(0, idx, dhc.view(nv, H))  # masked rows stay zero
        routes["gemm_compact"] = gemm_compact
    # the drop-in: whitened advantages as get_advantages_and_returns hands them to the loss
    mu, var = P.modeling.moments_to_mean_var(hp.adv_stats, unbiased=True)
    adv_w = ((hp.adv_raw.double() - mu) * torch.rsqrt(var + 1e-8)).float()
    hg = new_h.detach().clone().requires_grad_(True)
    wg = w.detach().clone().requires_grad_(True)
    vg = values.detach().clone().requires_grad_(True)
    lp_old, rets = hp.lp_old.clone(), hp.returns.clone()

    def dropin():
        hg.grad = wg.grad = vg.grad = None
        loss, _ = cfg.loss_from_hidden(hg, wg, vg, labels, lp_old, old_values, adv_w, rets, mask,
                                       return_device_stats=True)
        loss.backward()
    routes["dropin"] = dropin

    names = list(routes)
    for route in names + names:  # ~50 ms of load first: an idle chip runs slow (settle_and_warm)
        for _ in range(4):
            routes[route]()
    hp.wait_stats()
    torch.cuda.synchronize()
    times = {n: [] for n in names}
    for r in range(rounds):
        for route in names[r % len(names):] + names[:r % len(names)]:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(steps):
                routes[route]()
            hp.wait_stats()
            if hpc is not None:
                hpc.wait_stats()
            e1.record()
            torch.cuda.synchronize()
            times[route].append(e0.elapsed_time(e1) / steps)
    med = {n: sorted(v)[len(v) // 2] for n, v in times.items()}
    fused_ms = med["fused"]
    # the plan the library ran for this workspace: saved P = 3 MFMA passes (S and O forward,
    # dSᵀ·h from the stored P), recompute = 4 (S again in the dW kernel)
    savep = P._lib.query("trlx_ppo_loss_from_hidden_plan", B * T, H, V, hp.lm_loss_ws.numel()) == 1
    passes = 3 if savep else 4
    flop = passes * 2 * nv * V * H  # over the live tokens
    ach = flop / (fused_ms * 1e-3) / 1e12
    out = {"shape": {"rows": B, "seq_len": T, "vocab": V, "hidden": H, "tokens": B * T, "live_tokens": nv,
                     "masked": masked},
           **{f"{n}_ms_per_update": round(v, 4) for n, v in med.items()},
           "fused_vs_gemm": round(med["gemm"] / fused_ms, 4),
           **({"fused_vs_gemm_compact": round(med["gemm_compact"] / fused_ms, 4)} if "gemm_compact" in med else {}),
           "dropin_vs_fused": round(med["dropin"] / fused_ms, 4),
           "ratios_note": ("fused_vs_gemm_compact is the kernel comparison (both routes over the live tokens); "
                           "fused_vs_gemm also counts the masked tokens the reference's structure multiplies"
                           if masked else "every token live: fused_vs_gemm is the kernel comparison"),
           "rounds_ms": {k: [round(v, 4) for v in vs] for k, vs in times.items()},
           "roofline": {"bound": "mfma", "achieved": round(ach, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(ach / MFMA_BF16_PEAK_TFLOPS, 4), "flop_per_update": flop,
                        "mfma_passes": passes, "plan": "saved_p" if savep else "recompute",
                        "note": "N·V·H multiply-add passes over the live tokens per fused update — saved P: S and "
                                "O = P·W forward, dSᵀ·h from the stored bf16 P (the reference's three GEMMs' "
                                "count); recompute: + S again in the dW kernel (combine, compaction and loss "
                                "tail included in the time)"},
           "steps_per_round": steps, "rounds": rounds}
    del hp, hpc, h, w, ref_h, new_h, hg, wg, vg
    torch.cuda.empty_cache()
    return out


SETTLE_CHUNK = 8  # steps between the ranks' agreement on whether the settle is over (N > 1)


def settle_and_warm(step, torch, args, dev, world=1, dist=None):
    """The W warm-up steps, then (settle) more steps until the GPU has been kept busy for
    --settle-ms.  Measured cause (tools/slowstart_probe.py, profiles/r02_slowstart.log): after
    an idle period (process start, or 1 s of sleep) this step runs 10-20 % slow for its first
    ~20-40 ms of sustained load, the read-only experience launch most (244 -> 196 us), whatever
    the buffers — a chip power/clock state, not first touch.  The queue is kept at most
    4 steps deep (fence-free events) so the wall clock of the settle is GPU-busy time.
    N > 1: every step carries collectives, so every rank must run the SAME number of settle
    steps (one extra step on one rank pairs its all-reduces with the next step's of the
    others and leaves its last one waiting forever): the ranks decide together, every
    SETTLE_CHUNK steps, with an all-reduce of their "settled" flags (MIN: until all are)."""
    from trlx_t5_amd.timing import LaunchEvent
    t0 = time.perf_counter()
    for _ in range(args.warmup):
        step()
    extra = 0
    if args.settle_ms > 0:
        ring = [LaunchEvent() for _ in range(4)]
        s = torch.cuda.current_stream(dev)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        flag = torch.zeros(1, dtype=torch.int32) if world > 1 else None
        while extra < SETTLE_MAX_STEPS:
            if world > 1:
                if extra % SETTLE_CHUNK == 0:
                    flag[0] = int((time.perf_counter() - t1) * 1e3 >= args.settle_ms)
                    f = flag.to(dev)
                    dist.all_reduce(f, dist.ReduceOp.MIN)  # the same decision on every rank
                    if int(f.item()):
                        break
            elif (time.perf_counter() - t1) * 1e3 >= args.settle_ms:
                break
            step()
            ev = ring[extra % len(ring)]
            ev.record(s)
            extra += 1
            if extra >= len(ring):  # wait for the step recorded 3 steps earlier
                ring[extra % len(ring)].synchronize()
    torch.cuda.synchronize()
    return args.warmup + extra, (time.perf_counter() - t0) * 1e3


def timed_run(step, hp, torch, dist, args, dev, world, names):
    """Exactly K steps between barrier + synchronize pairs; max over ranks.  Per-kernel HIP
    events (fence-free) on every TIMER_EVERY-th step, around the vocab-row launches only:
    an event between two kernels idles the queue briefly, so instrumenting every step
    would tax `value`."""
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timers = {}
    hp.timer_names = names
    t0 = time.perf_counter()
    for i in range(args.steps):
        hp.timers = timers if (not args.no_timers and i % TIMER_EVERY == TIMER_EVERY - 1) else None
        step()
    hp.timers = None
    if hasattr(hp, "wait_stats"):
        hp.wait_stats()  # a deferred loss tail runs here, inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    per_rank = [elapsed]
    if world > 1:  # every rank's own clock (the spread says whether one rank held the others)
        t = torch.zeros(world, dtype=torch.float64, device=dev)
        t[dist.get_rank()] = elapsed
        dist.all_reduce(t, dist.ReduceOp.SUM)
        per_rank = t.tolist()
        elapsed = max(per_rank)
    kern_ms, samples = {}, {}
    for name, evs in timers.items():  # HIP events on the launch stream, timed region only
        kern_ms[name] = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
        samples[name] = len(evs)
    return elapsed, kern_ms, samples, per_rank


def pmc_traffic(key, dom):
    """HBM bytes per launch from the committed rocprofv3 PMC passes (not measured by this run:
    PMC needs its own rocprofv3 passes) and where they came from."""
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(pmc):
        return None, None
    with open(pmc) as f:
        rec = json.load(f)
    val = rec.get(key, {}).get(dom)
    if val is None:
        return None, None
    meta = rec.get("_meta", {}).get(key, {})
    src = (f"profiles/pmc_traffic.json[{key}][{dom}]: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes "
           f"(FETCH x2, MI355X_MICROARCH.md §HBM) at commit {meta.get('commit', 'unrecorded')}"
           f"{', ' + meta['command'] if 'command' in meta else ''}; not measured by this run")
    return val, src


def roofline(kern_ms, samples, ab, tokens, doms, elapsed, steps, traffic_key):
    if not kern_ms:
        return None
    dom = max(doms, key=lambda k: kern_ms.get(k, 0.0))
    ach = ab[dom] * tokens / (kern_ms[dom] * 1e-3) / 1e9
    traffic, src = pmc_traffic(traffic_key, dom) if traffic_key else (None, None)
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": src, "kernel": dom,
            "bytes_per_launch": int(round(ab[dom] * tokens)), "avg_launch_us": round(kern_ms[dom] * 1e3, 2),
            "timer_samples": samples.get(dom, 0),
            "kernels_avg_us": {k: round(v * 1e3, 2) for k, v in kern_ms.items()},
            "step_frac": round(ab["step"] * tokens / (elapsed / steps) / 1e9 / HBM_PEAK_GBS, 4)}


def ppo_setup(torch, P, args, B, T, V, dev, rank, masked, ldt, world=1, comm=None):
    x = make_inputs(torch, B, T, V, dev, seed=1000 + rank, masked=masked, dtype=ldt)
    cfg = P.PPOConfig()  # configs/ppo_config.yml method: adaptive KL (target 6, horizon 10000), clip 10
    ctl = None if args.host_state else P.PPOControlState.from_config(cfg, dev, n_steps=B)  # train.batch_size per process
    pipelined = args.schedule in ("pipelined", "auto")
    defer = not (args.overlap_tail or args.no_defer_tail)  # pipelined too: split beta keeps its tail foldable
    hp = P.PPOHotPath(cfg, B, T, V, ldt, dev, kl_coef=0.05, ctl=ctl, overlap_tail=args.overlap_tail,
                      loss_norm=args.loss_norm, defer_tail=defer, comm=comm, split_beta=args.split_beta)
    hp._fold_gae = not args.no_gae_fold
    hp._derive_coef = not args.coef_launch
    fn = hp.pipeline_step if pipelined else hp.step  # pipelined: each call = E rows of one batch + loss of the last

    def step():
        return fn(x["logits"], x["ref_logits"], x["new_logits"], x["labels"], x["old_values"], x["values"],
                  x["scores"], lengths=x["lengths"], mask=x["mask"])
    return hp, step, x


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.rank_timeout))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}: refusing a mislabelled run")
    if args.dry_run:
        return dry_run(args)
    import torch
    import torch.distributed as dist
    import __graft_entry__
    P = __graft_entry__.load_package()
    P.load_library()
    for kv in args.tune:
        k, v = kv.split("=")
        P._lib.set_tuning(k, int(v))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    use_dist = world > 1 or args.dist
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        kw = dict(rank=rank, world_size=world)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, **kw)
        else:
            dist.init_process_group("gloo", **kw)
    comm, comm_kind = None, ("torch" if use_dist else None)
    if use_dist and args.backend == "nccl" and args.comm != "torch" and args.config != "c5":
        try:
            comm = P.RcclComm.from_process_group(device=dev)
            comm_kind = "rccl"
        except Exception as e:  # auto: keep torch.distributed; rccl: explicit request, fail loudly
            if args.comm == "rccl":
                raise
            print(f"warning: RCCL helper unavailable ({e}); using torch.distributed collectives", file=sys.stderr)

    B, T, V, desc = resolve_shape(args, world)
    if args.logits_dtype == "fp32" and args.config != "c5":
        desc = desc.replace("bf16 logits", "fp32 logits") + ("" if "logits" in desc else ", fp32 logits")
    ilql = args.config == "c5"
    masked = args.config == "c3"
    if ilql:
        lg, qs, tqs, vs, batch = make_ilql_inputs(torch, P, B, T, V, dev, seed=1000 + rank)
        hp = P.ILQLHotPath(P.ILQLConfig(), B, T, V, torch.float32, dev)

        def step():
            return hp.step(lg, qs, tqs, vs, batch)
        names = {"rows"}
        tokens = B * (T - 1)  # action tokens; per-launch bytes of the rows kernel
        ab = {"rows": ilql_algorithmic_bytes(B, T, V, 4) / tokens}
        ab["step"] = ab["rows"]
        doms = ("rows",)
        traffic_key = None if args.global_batch else "c5"
        schedule = "serial"
    else:
        ldt = torch.float32 if args.logits_dtype == "fp32" else torch.bfloat16
        hp, step, x = ppo_setup(torch, P, args, B, T, V, dev, rank, masked, ldt, world, comm)
        schedule = "pipelined" if args.schedule in ("pipelined", "auto") else "serial"
        names = {"experience", "loss"}
        tokens = B * T
        # ragged batch (C3): the share of positions inside their rollout's decoder length
        fill = float(x["lengths"].sum().item()) / tokens if masked else 1.0
        ab = algorithmic_bytes(V, 4 if args.logits_dtype == "fp32" else 2, masked, schedule == "pipelined", fill)
        doms = ("experience", "loss")
        # PMC bytes were collected at the config's rows per GPU
        traffic_key = None if args.global_batch else args.config + ("_fp32" if args.logits_dtype == "fp32" else "")

    warm_steps, warm_ms = settle_and_warm(step, torch, args, dev, world, dist)
    elapsed, kern_ms, samples, per_rank = timed_run(step, hp, torch, dist, args, dev, world, names)
    roof = roofline(kern_ms, samples, ab, tokens, doms, elapsed, args.steps, traffic_key)

    # Secondary line (C2 at N=1): the same step with fp32 logits (the reference's GPT path,
    # ppo_models.py:225-289; BASELINE.md asks for both dtypes), same K / W / settle.
    fp32_line = None
    if (not ilql and world == 1 and args.config == "c2" and args.logits_dtype == "bf16" and not args.no_fp32_line
            and not args.global_batch):
        del hp, step, x
        torch.cuda.empty_cache()
        hp32, step32, x32 = ppo_setup(torch, P, args, B, T, V, dev, rank, masked, torch.float32, world, comm)
        w32, wms32 = settle_and_warm(step32, torch, args, dev)
        el32, km32, sm32, _ = timed_run(step32, hp32, torch, dist, args, dev, world, names)
        fp32_line = {"value": round(tokens * args.steps / el32, 1), "unit": "tokens/s",
                     "ms_per_step": round(el32 / args.steps * 1e3, 4), "warmup_steps_run": w32,
                     "warmup_ms": round(wms32, 1),
                     "roofline": roofline(km32, sm32, algorithmic_bytes(V, 4, masked, schedule == "pipelined"), tokens, doms, el32,
                                          args.steps, "c2_fp32")}
        del hp32, step32, x32
        torch.cuda.empty_cache()

    # Secondary line (C2 at N=1): §8f-2's loss side from hidden states (the fused
    # route's speed-up over the hipBLASLt logits route, measured by the driver's run)
    from_hidden = None
    if (not ilql and world == 1 and args.config == "c2" and args.logits_dtype == "bf16" and not args.no_from_hidden
            and not args.global_batch):
        from_hidden = {name: from_hidden_leg(torch, P, dev, name, args.from_hidden_steps)
                       for name in FROM_HIDDEN_SHAPES}

    out = None
    if rank == 0:
        cpu = None
        if world == 1 and args.cpu_seconds > 0:
            if ilql:
                cpu = ilql_cpu_baseline(torch, T, V, args.cpu_seconds)
            else:  # both logits dtypes; `cpu_baseline` itself is the one matching this line
                by = {n: cpu_baseline(torch, T, V, args.cpu_seconds, d)
                      for n, d in (("bf16", torch.bfloat16), ("fp32", torch.float32))}
                cpu = dict(by[args.logits_dtype])
                cpu["by_logits_dtype"] = {n: {k: (round(v, 1) if k == "value" else v) for k, v in c.items()
                                              if k in ("value", "sample")} for n, c in by.items()}
        ms = elapsed / args.steps * 1e3
        out = {
            "metric": METRIC_ILQL if ilql else METRIC,
            "value": round(world * tokens * args.steps / elapsed, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_steps_run": warm_steps,
            "warmup_ms": round(warm_ms, 1),
            "settle_ms": args.settle_ms,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.global_batch else "weak",
            "vs_baseline": None,
            "dtype": "f32",  # arithmetic type; logits_dtype in config
            "data": "synthetic",
            "config": {"workload": desc, "rows_per_gpu": B, "global_batch": B * world, "seq_len": T, "vocab": V,
                       "logits_dtype": "fp32" if ilql else args.logits_dtype, "tokens_per_gpu_step": tokens,
                       "parallelism": f"dp{world}", "schedule": schedule, "comm": comm_kind,
                       "comm_nranks": comm.nranks if comm is not None else (world if use_dist else None)},
            "rank_ms_per_step": {"min": round(min(per_rank) / args.steps * 1e3, 4),
                                 "max": round(max(per_rank) / args.steps * 1e3, 4), "ranks": len(per_rank)},
            **({"ragged": {"valid_token_fraction": round(fill, 4),
                           "note": "tokens counts every decoder position of the padded batch; logits rows past a "
                                   "rollout's length are store padding (lp = 0) and masked loss rows have zero "
                                   "gradient, so neither is read (roofline bytes count only the rows read)"}}
               if masked and not ilql else {}),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if fp32_line:
            out["fp32_logits"] = fp32_line
        if from_hidden:
            out["from_hidden"] = from_hidden
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.barrier()
        if comm is not None:
            torch.cuda.synchronize(dev)
            comm.close()
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
