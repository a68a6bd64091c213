"""Worker functions for spawned torch.distributed (gloo) test processes.  Importable in
a fresh child: it registers the package itself."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()

import torch  # noqa: E402

from trlx_t5_amd.modeling import _allreduce_moments, moments_to_mean_var  # noqa: E402


def whiten_stats_worker(rank, world, port, xs, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shard = xs.chunk(world, dim=0)[rank].double()
    st = torch.stack([shard.sum(), (shard * shard).sum(), torch.tensor(float(shard.numel())),
                      torch.tensor(0.0, dtype=torch.float64)])
    _allreduce_moments(st)  # the product's exchange: ONE all-reduce of {sum, sumsq, n}
    mean, var = moments_to_mean_var(st, unbiased=False)
    q.put((rank, float(mean), float(var), float(st[2])))
    dist.barrier()
    dist.destroy_process_group()


def hot_path_step_worker(rank, world, port, inputs, q, loss_norm="rank", mode="step", cfg_kwargs=None):
    """One rank of a DP PPO step on cuda:0 over gloo (the product's exchange: the whitening
    record all-reduce inside PPOHotPath.experience).  Rank r takes the contiguous row block
    r of the batch (accelerate_ppo_model.py:146-148 sharding)."""
    import torch.distributed as dist
    import trlx_t5_amd as P
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    sh = {k: (v.chunk(world, dim=0)[rank].contiguous().to(dev) if v is not None else None) for k, v in inputs.items()}
    B, T, V = sh["logits"].shape
    hp = P.PPOHotPath(P.PPOConfig(**(cfg_kwargs or {})), B, T, V, torch.bfloat16, dev, kl_coef=0.05,
                      loss_norm=loss_norm)
    args = (sh["logits"], sh["ref_logits"], sh["new_logits"], sh["labels"], sh["old_values"], sh["values"],
            sh["scores"])
    if mode == "pipelined":  # split-beta schedule: one batch through pipeline_step + flush
        assert hp.pipeline_step(*args, lengths=sh["lengths"], mask=sh["mask"]) is None
        loss, stats, dlogits, dvalues = hp.pipeline_flush()
    else:
        loss, stats, dlogits, dvalues = hp.step(*args, lengths=sh["lengths"], mask=sh["mask"])
    hp.wait_stats()
    torch.cuda.synchronize()
    q.put((rank, {"lp": hp.lp_old.cpu(), "rewards": hp.rewards.cpu(), "adv_stats": hp.adv_stats.cpu(),
                  "loss": loss.cpu(), "dlogits": dlogits.float().cpu(), "dvalues": dvalues.cpu(),
                  "stats": stats.cpu(), "returns": hp.returns.cpu(), "adv_raw": hp.adv_raw.cpu()}))
    dist.barrier()
    dist.destroy_process_group()


def ctl_step_worker(rank, world, port, inputs, scores_seq, scale, q):
    """Two DP steps with the device controller state: the score moments are all-reduced
    (get_global_statistics semantics for RunningMoments), ref stats stay rank-local
    (scores.std() of the rank's chunk, ppo_orchestrator.py:96-98)."""
    import torch.distributed as dist
    import trlx_t5_amd as P
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    sh = {k: (v.chunk(world, dim=0)[rank].contiguous().to(dev) if v is not None else None) for k, v in inputs.items()}
    B, T, V = sh["logits"].shape
    cfg = P.PPOConfig(scale_reward=scale, cliprange_reward=10)
    ctl = P.PPOControlState.from_config(cfg, dev, n_steps=B)
    hp = P.PPOHotPath(cfg, B, T, V, torch.bfloat16, dev, kl_coef=0.0, ctl=ctl)
    out = []
    for s in scores_seq:
        hp.step(sh["logits"], sh["ref_logits"], sh["new_logits"], sh["labels"], sh["old_values"], sh["values"],
                s.chunk(world)[rank].contiguous().to(dev))
        torch.cuda.synchronize()
        out.append({"rewards": hp.rewards.cpu(), "state": ctl.host(), "approx_kl": float(hp.stats[8])})
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def drop_in_surface_worker(rank, world, port, xs_all, q):
    """The drop-in distributed surface on cuda:0 under an initialised gloo group, exactly as
    the reference's golden generator calls it (tests/golden/make_golden.py _dist_worker):
    get_global_statistics / whiten / whiten(shift_mean=False) on the rank's chunk, plus
    RunningMoments.update (modeling.py:83-104, dist branch)."""
    import torch.distributed as dist
    import trlx_t5_amd as P
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    res = {}
    for key, xs in xs_all.items():
        shard = xs.chunk(world, dim=0)[rank].contiguous().to(dev)
        mean, var, count = P.get_global_statistics(shard)
        w = P.whiten(shard)
        w2 = P.whiten(shard, shift_mean=False)
        wl = P.whiten(shard, distributed=False)  # the var_mean branch even with the group up
        rm = P.RunningMoments()
        bm, bs = rm.update(shard.float())
        res[key] = {"mean": float(mean), "var": float(var), "count": float(count), "dtype": str(mean.dtype),
                    # numpy (pickled by value): a torch CPU tensor would travel as a shared-memory
                    # fd that dies with this process
                    "whiten": w.float().cpu().numpy(), "whiten_noshift": w2.float().cpu().numpy(),
                    "whiten_local": wl.float().cpu().numpy(),
                    "rm": (float(rm.mean), float(rm.var), float(rm.std), float(rm.count), float(bm), float(bs))}
    torch.cuda.synchronize()
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def pipeline_worker(rank, world, port, batches, q, use_ctl, overlap, loss_norm="rank", scale="running"):
    """The same sequence of batches through PPOHotPath.step (serial) and
    PPOHotPath.pipeline_step (experience of batch k+1 ahead of the loss of batch k, the
    whitening all-reduce in flight meanwhile) on this rank's row shards.  Returns every
    batch's outputs of both schedules (numpy, pickled by value)."""
    import torch.distributed as dist
    import trlx_t5_amd as P
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    shards = [{k: (v.chunk(world, dim=0)[rank].contiguous().to(dev) if v is not None else None)
               for k, v in b.items()} for b in batches]
    B, T, V = shards[0]["logits"].shape
    res = {}
    for mode in ("serial", "pipelined", "unsplit"):
        cfg = P.PPOConfig(scale_reward=scale)
        ctl = P.PPOControlState.from_config(cfg, dev, n_steps=B) if use_ctl else None
        # scale False / "ref": pipeline_step merges each batch's score moments one batch late
        # (lag), the final controller state is still the serial one
        # "serial": step() with the split-beta kernels pipeline_step uses (bit-identical);
        # "unsplit": the default step() kernels (equal up to fp32 association); defer the
        # loss tails unless the side-stream tail is under test
        hp = P.PPOHotPath(cfg, B, T, V, torch.bfloat16, dev, kl_coef=0.05, ctl=ctl, overlap_tail=overlap,
                          defer_tail=not overlap, split_beta=mode != "unsplit", loss_norm=loss_norm)
        outs = []

        def grab(o):
            loss, stats, dl, dv = o
            hp.wait_stats()
            torch.cuda.synchronize()
            outs.append([loss.cpu().numpy(), stats.cpu().numpy(), dl.float().cpu().numpy(), dv.cpu().numpy(),
                         hp.rewards.cpu().numpy(), hp.returns.cpu().numpy()])

        for sh in shards:
            args = (sh["logits"], sh["ref_logits"], sh["new_logits"], sh["labels"], sh["old_values"], sh["values"],
                    sh["scores"])
            if mode != "pipelined":
                grab(hp.step(*args, lengths=sh["lengths"], mask=sh["mask"]))
            else:
                o = hp.pipeline_step(*args, lengths=sh["lengths"], mask=sh["mask"])
                if o is not None:
                    grab(o)
        if mode == "pipelined":
            grab(hp.pipeline_flush())
        # the controller state is compared after the last batch: mid-sequence snapshots differ
        # by design (the pipelined schedule has already run batch k+1's GAE tail, which
        # advances RunningMoments, when batch k's loss is returned)
        hp.wait_stats()
        torch.cuda.synchronize()
        res[mode] = (outs, ctl.state.cpu().numpy() if use_ctl else None)
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def rccl_world1_worker(port, inputs, xs_all, q):
    """torch.distributed with the "nccl" backend (= RCCL on ROCm) at world size 1, on cuda:0:
    the product's exchange path for real — ProcessGroupNCCL init with device_id, the async
    whitening all-reduce + stream wait of pipeline_step, the blocking one of step(), and the
    drop-in get_global_statistics / whiten / RunningMoments."""
    import torch.distributed as dist
    import trlx_t5_amd as P
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    x = {k: (v.to(dev) if v is not None else None) for k, v in inputs[0].items()}
    B, T, V = x["logits"].shape
    res = {"backend": dist.get_backend()}
    comm = P.RcclComm.from_process_group(device=dev)
    v = torch.randn(5, dtype=torch.float64, device=dev)
    w = comm.allreduce_(v.clone())
    torch.cuda.synchronize()
    res["comm_identity"] = bool(torch.equal(v, w))
    try:
        comm.allreduce_(v.float())
        res["comm_rejects_f32"] = False
    except ValueError:
        res["comm_rejects_f32"] = True
    for mode, kind in (("serial", "torch"), ("pipelined", "torch"), ("serial", "rccl"), ("pipelined", "rccl"),
                       ("unsplit", "rccl")):
        cfg = P.PPOConfig()
        ctl = P.PPOControlState.from_config(cfg, dev, n_steps=B)
        hp = P.PPOHotPath(cfg, B, T, V, torch.bfloat16, dev, kl_coef=0.05, ctl=ctl,
                          comm=comm if kind == "rccl" else None, split_beta=mode != "unsplit")
        outs = []
        for b in inputs:
            xb = {k: (v.to(dev) if v is not None else None) for k, v in b.items()}
            args = (xb["logits"], xb["ref_logits"], xb["new_logits"], xb["labels"], xb["old_values"], xb["values"],
                    xb["scores"])
            o = hp.step(*args) if mode != "pipelined" else hp.pipeline_step(*args)
            if o is not None:
                torch.cuda.synchronize()
                outs.append([t.float().cpu().numpy() for t in o])
        if mode == "pipelined":
            o = hp.pipeline_flush()
            torch.cuda.synchronize()
            outs.append([t.float().cpu().numpy() for t in o])
        torch.cuda.synchronize()
        res[(mode, kind)] = (outs, hp.adv_stats.cpu().numpy(), ctl.state.cpu().numpy())
    comm.close()
    surf = {}
    for key, xs in xs_all.items():
        xd = xs.to(dev)
        mean, var, count = P.get_global_statistics(xd)
        surf[key] = (float(mean), float(var), float(count), P.whiten(xd).float().cpu().numpy(),
                     P.whiten(xd, shift_mean=False).float().cpu().numpy())
    res["surface"] = surf
    q.put(res)
    dist.barrier()
    dist.destroy_process_group()


def rccl_scores_reuse_worker(port, inputs, q):
    """under the lag schedule the side stream's moments kernel reads the
    caller's `scores` after pipeline_step returns.  Each batch's scores are a fresh tensor
    dropped right after the call, and a same-sized tensor allocated at once and filled with
    NaN on the main stream (the caching allocator hands it the freed block unless the side
    stream's use was recorded).  The controller state must equal the serial schedule's."""
    import torch.distributed as dist
    import trlx_t5_amd as P
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    comm = P.RcclComm.from_process_group(device=dev)
    res = {}
    for mode in ("serial", "pipelined"):
        cfg = P.PPOConfig(scale_reward=False)  # lag: the moments ride the side stream
        B, T, V = inputs[0]["logits"].shape
        ctl = P.PPOControlState.from_config(cfg, dev, n_steps=B)
        hp = P.PPOHotPath(cfg, B, T, V, torch.bfloat16, dev, kl_coef=0.05, ctl=ctl, comm=comm, split_beta=True,
                          defer_tail=True)
        fixed = [{k: v.to(dev) for k, v in b.items() if k != "scores"} for b in inputs]
        poison = []
        for b, xb in zip(inputs, fixed):
            sc = b["scores"].to(dev)  # a fresh allocation per batch
            args = (xb["logits"], xb["ref_logits"], xb["new_logits"], xb["labels"], xb["old_values"], xb["values"], sc)
            if mode == "pipelined":
                hp.pipeline_step(*args)
                assert hp._lag, "the test needs the lag schedule"
            else:
                hp.step(*args)
            del sc, args
            p = torch.empty(B, dtype=torch.float32, device=dev)  # the freed block, if nothing held it
            p.fill_(float("nan"))
            poison.append(p)
        if mode == "pipelined":
            hp.pipeline_flush()
        hp.wait_stats()
        torch.cuda.synchronize()
        res[mode] = ctl.state.cpu().numpy()
    comm.close()
    q.put(res)
    dist.barrier()
    dist.destroy_process_group()


def pipeline_hidden_worker(rank, world, port, batches, q, loss_norm="rank", use_ctl=False):
    """§8f-2 under the data-parallel schedule: the same batches through step_from_hidden (serial,
    split beta) and pipeline_step_from_hidden (the lm_head experience of batch k+1 ahead of the
    loss side of batch k, the whitening all-reduce of batch k in flight meanwhile) on this
    rank's contiguous row shards (accelerate_ppo_model.py:146-148).  Returns every batch's
    outputs of both schedules (numpy, pickled by value)."""
    import torch.distributed as dist
    import trlx_t5_amd as P
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    shards = [{k: (v.chunk(world, dim=0)[rank].contiguous().to(dev) if v is not None and k != "w" else
                   (v.to(dev) if v is not None else None)) for k, v in b.items()} for b in batches]
    B, T, _ = shards[0]["h"].shape
    V = shards[0]["w"].shape[0]
    res = {}
    for mode in ("serial", "pipelined"):
        cfg = P.PPOConfig()
        ctl = P.PPOControlState.from_config(cfg, dev, n_steps=B) if use_ctl else None
        hp = P.PPOHotPath(cfg, B, T, V, torch.bfloat16, dev, kl_coef=0.05, ctl=ctl, defer_tail=True, split_beta=True,
                          loss_norm=loss_norm)
        outs = []

        def grab(o):
            loss, stats, dh, dw, dv = o
            hp.wait_stats()
            torch.cuda.synchronize()
            outs.append([loss.cpu().numpy(), stats.cpu().numpy(), dh.float().cpu().numpy(), dw.float().cpu().numpy(),
                         dv.cpu().numpy(), hp.rewards.cpu().numpy(), hp.returns.cpu().numpy()])

        for sh in shards:
            args = (sh["h"], sh["w"], sh["ref_h"], sh["w"], sh["new_h"], sh["labels"], sh["old_values"], sh["values"],
                    sh["scores"])
            kw = dict(lengths=sh["lengths"], mask=sh["mask"], route="fused", loss_route="fused")
            if mode == "serial":
                grab(hp.step_from_hidden(*args, **kw))
            else:
                o = hp.pipeline_step_from_hidden(*args, **kw)
                if o is not None:
                    grab(o)
        if mode == "pipelined":
            grab(hp.pipeline_flush())
        hp.wait_stats()
        torch.cuda.synchronize()
        res[mode] = (outs, ctl.state.cpu().numpy() if use_ctl else None)
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()
