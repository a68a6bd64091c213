"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Container-only script (needs /root/reference, which never travels to the GPU box).
It imports the reference's hot-path files standalone (`import trlx`
fails on absent deps, but the individual files load once their package shells and
an annotation-only `torchtyping` stub are registered), runs them on seeded synthetic
inputs and writes inputs + outputs as plain `.npz` data.  bf16 tensors are stored as
their raw uint16 bit patterns so the fixtures are exact.

Reference functions exercised (all file:line into /root/reference):
  trlx/utils/modeling.py:37-41   logprobs_from_logits        (+ autograd backward)
  trlx/utils/modeling.py:9-21    get_global_statistics       (gloo world 1/2/4)
  trlx/utils/modeling.py:24-34   whiten                      (non-dist unbiased, dist biased)
  trlx/utils/modeling.py:72-104  RunningMoments.update
  trlx/model/nn/ppo_models.py:26-58    Adaptive/FixedKLController
  trlx/model/nn/ppo_models.py:121-139  PPOConfig.get_advantages_and_returns
  trlx/model/nn/ppo_models.py:141-199  PPOConfig.loss         (+ autograd grads)
  trlx/orchestrator/ppo_orchestrator.py:96-112,163-167 (score prep + KL reward; that file
      imports ray, so its arithmetic is evaluated here with the reference's own ops,
      line for line, on the reference logprobs)
  trlx/model/nn/ilql_models.py:52-116  ILQLConfig.loss        (+ autograd grads)
  trlx/model/accelerate_ppo_model.py:18-25,63-76  shift_tokens_right / get_model_inputs

Run:  python tests/golden/make_golden.py      (writes tests/golden/*.npz)
"""
import importlib.util
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------- loader
def _shell(name):
    m = types.ModuleType(name)
    m.__path__ = []
    sys.modules[name] = m
    return m


def _load(modname, relpath):
    spec = importlib.util.spec_from_file_location(modname, os.path.join(REF, relpath))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    for p in ["trlx", "trlx.data", "trlx.utils", "trlx.model", "trlx.model.nn"]:
        _shell(p)
    tt = types.ModuleType("torchtyping")

    class _TT:
        def __class_getitem__(cls, item):
            return torch.Tensor

    tt.TensorType = _TT
    sys.modules["torchtyping"] = tt
    modeling = _load("trlx.utils.modeling", "trlx/utils/modeling.py")
    _load("trlx.data.method_configs", "trlx/data/method_configs.py")
    ilql_types = _load("trlx.data.ilql_types", "trlx/data/ilql_types.py")
    ppo_models = _load("trlx.model.nn.ppo_models", "trlx/model/nn/ppo_models.py")
    # ilql_models imports deepspeed / wandb at module scope; transformers must resolve
    # its own optional-dependency probes before those stubs exist.
    import transformers  # noqa: F401
    from transformers import AutoModelForCausalLM, PretrainedConfig  # noqa: F401

    sys.modules.setdefault("deepspeed", types.ModuleType("deepspeed"))
    sys.modules.setdefault("wandb", types.ModuleType("wandb"))
    ilql_models = _load("trlx.model.nn.ilql_models", "trlx/model/nn/ilql_models.py")
    return modeling, ppo_models, ilql_models, ilql_types


# --------------------------------------------------------------------------- helpers
def bf16_bits(t):
    return t.to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)


def store(t):
    """Tensor -> numpy: bf16 as raw uint16 bits, else native."""
    t = t.detach().cpu().clone()  # own copy: never alias a tensor that is later shared/modified
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16).copy()
    return t.numpy().copy()


def gen(seed):
    return torch.Generator().manual_seed(seed)


PPO_METHOD = dict(  # configs/ppo_config.yml:26-47 (the `method:` block)
    name="ppoconfig", num_rollouts=128, chunk_size=128, ppo_epochs=4, init_kl_coef=0.05,
    target=6, horizon=10000, gamma=1, lam=0.95, cliprange=0.2, cliprange_value=0.2,
    vf_coef=1, scale_reward=False, ref_mean=None, ref_std=None, cliprange_reward=10,
    gen_kwargs=dict(max_length=49, min_length=49, top_k=1, top_p=1, do_sample=True),
)


# --------------------------------------------------------------------------- A1
def make_lsm_gather(modeling):
    out = {}
    cases = [
        ("small_f32", 4, 6, 37, torch.float32, 1.0),
        ("small_bf16", 4, 6, 37, torch.bfloat16, 1.0),
        ("peaked_f32", 3, 5, 101, torch.float32, 4.0),
        ("wide50257_f32", 1, 2, 50257, torch.float32, 1.0),
        ("wide50257_bf16", 1, 3, 50257, torch.bfloat16, 1.0),
        ("wide32128_bf16", 1, 3, 32128, torch.bfloat16, 1.0),
    ]
    for name, B, T, V, dt, sigma in cases:
        g = gen(100 + len(out))
        x = torch.randn(B, T, V, generator=g) * sigma
        y = torch.randint(0, V, (B, T), generator=g)
        y[0, 0] = 0
        y[-1, -1] = V - 1
        if sigma > 1.0:  # "peaked" variant: +8 at the label
            x.scatter_add_(-1, y[..., None], torch.full((B, T, 1), 8.0))
        x = x.to(dt).requires_grad_(True)
        lp = modeling.logprobs_from_logits(x, y)
        w = torch.randn(B, T, generator=g).to(dt)
        (lp * w).sum().backward()
        out[f"{name}/logits"] = store(x)
        out[f"{name}/labels"] = y.numpy()
        out[f"{name}/lp"] = store(lp)
        out[f"{name}/w"] = store(w)
        out[f"{name}/dlogits"] = store(x.grad)
        out[f"{name}/dtype"] = np.array(str(dt))
    np.savez_compressed(os.path.join(OUT, "lsm_gather.npz"), **out)


# --------------------------------------------------------------------------- A2 + A7
def make_kl_reward(modeling):
    """ppo_orchestrator.py:96-112 (score prep) and :163-167 (KL-penalised reward),
    evaluated with the reference's own ops on reference logprobs."""
    out = {}
    for name, dt in [("f32", torch.float32), ("bf16", torch.bfloat16)]:
        g = gen(200 if dt == torch.float32 else 201)
        B, T, V = 6, 9, 53
        logits = torch.randn(B, T, V, generator=g).to(dt)
        ref_logits = (logits.float() + 0.1 * torch.randn(B, T, V, generator=g)).to(dt)
        resp = torch.randint(0, V, (B, T), generator=g)
        scores = torch.rand(B, generator=g) * 24 - 12  # U(-12, 12), some beyond the clip
        for mode in ["none", "running", "ref"]:
            running = modeling.RunningMoments()
            s = scores.clone()
            ref_mean, ref_std = s.mean(), s.std()          # :97-98
            m, sd = running.update(s)                     # :99
            if mode == "running":                         # :105-106
                s /= running.std
            elif mode == "ref":                           # :107-108
                s /= ref_std
            s = torch.clip(s, -10, 10)                    # :110-112
            lp = modeling.logprobs_from_logits(logits, resp)       # :154
            ref_lp = modeling.logprobs_from_logits(ref_logits, resp)  # :155
            kls = lp - ref_lp                              # :164
            beta = 0.05
            nsr = -beta * kls                              # :165
            rewards = nsr.clone()                          # :166
            rewards[:, -1] += s                            # :167
            k = f"{name}/{mode}"
            out[f"{k}/scores_in"] = scores.numpy()
            out[f"{k}/scores_out"] = s.numpy()
            out[f"{k}/batch_mean"] = np.array(float(m))
            out[f"{k}/batch_std"] = np.array(float(sd))
            out[f"{k}/running_mean"] = np.array(float(running.mean))
            out[f"{k}/running_std"] = np.array(float(running.std))
            out[f"{k}/lp"] = store(lp)
            out[f"{k}/ref_lp"] = store(ref_lp)
            out[f"{k}/rewards"] = store(rewards)
        out[f"{name}/logits"] = store(logits)
        out[f"{name}/ref_logits"] = store(ref_logits)
        out[f"{name}/labels"] = resp.numpy()
        out[f"{name}/beta"] = np.array(0.05)
    np.savez_compressed(os.path.join(OUT, "kl_reward.npz"), **out)


# --------------------------------------------------------------------------- A3/A4 (dist)
def _dist_worker(rank, world, port, xs_all, q):
    import torch.distributed as dist

    modeling, _, _, _ = load_reference()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    for key, xs in xs_all.items():
        shard = xs.chunk(world, dim=0)[rank].contiguous()
        mean, var, count = modeling.get_global_statistics(shard)
        w = modeling.whiten(shard)
        w2 = modeling.whiten(shard, shift_mean=False)
        res[key] = (float(mean), float(var), float(count), store(w), store(w2))
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, res))


def make_whiten(modeling):
    import torch.multiprocessing as mp

    out = {}
    xs_all = {}
    for name, dt, shape in [("f32", torch.float32, (8, 6)), ("bf16", torch.bfloat16, (8, 6)),
                            ("f32_big", torch.float32, (16, 48))]:
        g = gen(300 + len(xs_all))
        xs = (torch.randn(shape, generator=g) * 3 + 1.5).to(dt)
        xs_all[name] = xs
        out[f"{name}/xs"] = store(xs)
        out[f"{name}/nodist"] = store(modeling.whiten(xs))
        out[f"{name}/nodist_noshift"] = store(modeling.whiten(xs, shift_mean=False))
        out[f"{name}/nodist_disabled"] = store(modeling.whiten(xs, distributed=False))
    ctx = mp.get_context("spawn")
    for world in (1, 2, 4):
        q = ctx.Queue()
        port = 29600 + world
        procs = [ctx.Process(target=_dist_worker, args=(r, world, port, xs_all, q)) for r in range(world)]
        for p in procs:
            p.start()
        results = dict(q.get() for _ in range(world))
        for p in procs:
            p.join()
        for name in xs_all:
            m, v, c, _, _ = results[0][name]
            out[f"{name}/dist{world}/mean"] = np.array(m)
            out[f"{name}/dist{world}/var"] = np.array(v)
            out[f"{name}/dist{world}/count"] = np.array(c)
            out[f"{name}/dist{world}/whiten"] = np.concatenate([results[r][name][3] for r in range(world)])
            out[f"{name}/dist{world}/whiten_noshift"] = np.concatenate(
                [results[r][name][4] for r in range(world)])
    np.savez_compressed(os.path.join(OUT, "whiten.npz"), **out)


# --------------------------------------------------------------------------- A5
def make_gae(ppo_models):
    out = {}
    i = 0
    for T in (9, 48, 128):
        for gamma in (1.0, 0.99):
            for dt in (torch.float32, torch.bfloat16):
                for whit in (True, False):
                    cfg = ppo_models.PPOConfig.from_dict(dict(PPO_METHOD, gamma=gamma))
                    g = gen(400 + i)
                    B = 5
                    values = torch.randn(B, T, generator=g).to(dt)
                    rewards = (0.05 * torch.randn(B, T, generator=g)).to(dt)
                    rewards[:, -1] += 3.0
                    # zero right-padding (ppo_pipeline.py:47-65) on two rows
                    L = torch.tensor([T, max(1, T // 2), 1, T, T - 1])
                    pad = torch.arange(T)[None, :] >= L[:, None]
                    values[pad] = 0
                    rewards[pad] = 0
                    adv, ret = cfg.get_advantages_and_returns(values, rewards, T, use_whitening=whit)
                    k = f"T{T}_g{gamma}_{str(dt).split('.')[-1]}_w{int(whit)}"
                    out[f"{k}/values"] = store(values)
                    out[f"{k}/rewards"] = store(rewards)
                    out[f"{k}/lengths"] = L.numpy()
                    out[f"{k}/adv"] = store(adv)
                    out[f"{k}/ret"] = store(ret)
                    out[f"{k}/gamma"] = np.array(gamma)
                    out[f"{k}/lam"] = np.array(0.95)
                    i += 1
    np.savez_compressed(os.path.join(OUT, "gae.npz"), **out)


# --------------------------------------------------------------------------- A6 (+A1 bwd through A6)
def make_ppo_loss(ppo_models, modeling):
    out = {}
    cases = ["random", "masked", "ties", "wide_ratio", "bf16", "vf_coef"]
    for ci, name in enumerate(cases):
        g = gen(500 + ci)
        B, T = 4, 7
        dt = torch.bfloat16 if name == "bf16" else torch.float32
        cfg = ppo_models.PPOConfig.from_dict(dict(PPO_METHOD, vf_coef=(1.2 if name == "vf_coef" else 1)))
        lp = -torch.rand(B, T, generator=g) * 5
        olp = lp + 0.05 * torch.randn(B, T, generator=g)
        if name == "wide_ratio":
            olp = lp + 0.6 * torch.randn(B, T, generator=g)
        v = torch.randn(B, T, generator=g)
        ov = v + 0.3 * torch.randn(B, T, generator=g)
        adv = torch.randn(B, T, generator=g)
        ret = v + torch.randn(B, T, generator=g)
        mask = torch.ones(B, T, dtype=torch.long)
        if name == "masked":
            L = torch.tensor([7, 3, 1, 5])
            mask = (torch.arange(T)[None, :] < L[:, None]).long()
        if name == "ties":
            # values exactly on the clip bound (clamp passes the gradient at inclusive
            # bounds, torch.max splits ties 1/2-1/2); ratio == 1 exactly where lp == olp
            v[0, :] = ov[0, :] + 0.2
            v[1, :] = ov[1, :] - 0.2
            olp[2, :] = lp[2, :]
            adv[3, :3] = 0.0
        lp, olp, v, ov, adv, ret = (t.to(dt) for t in (lp, olp, v, ov, adv, ret))
        lp_ = lp.clone().requires_grad_(True)
        v_ = v.clone().requires_grad_(True)
        loss, stats = cfg.loss(lp_, v_, olp, ov, adv, ret, mask)
        loss.backward()
        k = name
        for nm, t in [("lp", lp), ("olp", olp), ("v", v), ("ov", ov), ("adv", adv), ("ret", ret)]:
            out[f"{k}/{nm}"] = store(t)
        out[f"{k}/mask"] = mask.numpy()
        out[f"{k}/vf_coef"] = np.array(float(cfg.vf_coef))
        out[f"{k}/loss"] = store(loss.detach().reshape(()))
        out[f"{k}/grad_lp"] = store(lp_.grad)
        out[f"{k}/grad_v"] = store(v_.grad)
        for sk, sv in stats.items():
            out[f"{k}/stats/{sk}"] = np.array(float(sv))
    # A1 backward through A6: logits -> logprobs -> PPO loss -> dlogits
    g = gen(550)
    B, T, V = 3, 5, 67
    cfg = ppo_models.PPOConfig.from_dict(PPO_METHOD)
    for dt in (torch.float32, torch.bfloat16):
        logits = torch.randn(B, T, V, generator=g).to(dt).requires_grad_(True)
        labels = torch.randint(0, V, (B, T), generator=g)
        lp = modeling.logprobs_from_logits(logits, labels)
        olp = (lp.detach().float() + 0.1 * torch.randn(B, T, generator=g)).to(dt)
        v = torch.randn(B, T, generator=g).to(dt).requires_grad_(True)
        ov = (v.detach().float() + 0.3 * torch.randn(B, T, generator=g)).to(dt)
        adv = torch.randn(B, T, generator=g).to(dt)
        ret = (v.detach().float() + torch.randn(B, T, generator=g)).to(dt)
        mask = torch.ones(B, T, dtype=torch.long)
        loss, stats = cfg.loss(lp, v, olp, ov, adv, ret, mask)
        loss.backward()
        k = "chain_" + str(dt).split(".")[-1]
        out[f"{k}/logits"] = store(logits)
        out[f"{k}/labels"] = labels.numpy()
        for nm, t in [("olp", olp), ("ov", ov), ("adv", adv), ("ret", ret), ("v", v)]:
            out[f"{k}/{nm}"] = store(t)
        out[f"{k}/loss"] = store(loss.detach().reshape(()))
        out[f"{k}/dlogits"] = store(logits.grad)
        out[f"{k}/grad_v"] = store(v.grad)
    np.savez_compressed(os.path.join(OUT, "ppo_loss.npz"), **out)


# --------------------------------------------------------------------------- A7 / A8
def make_host_state(modeling, ppo_models):
    out = {}
    # RunningMoments on the reference's own KAT inputs (tests/test_ppo.py:49-66)
    m = modeling.RunningMoments()
    arrs = [torch.arange(100, dtype=float), torch.ones(100, dtype=float),
            torch.exp(torch.arange(10, dtype=float)), torch.tensor([-10, -1, 0, 1, 10], dtype=float)]
    for i, a in enumerate(arrs):
        bm, bs = m.update(a)
        out[f"rm/{i}/in"] = a.numpy()
        out[f"rm/{i}/batch_mean"] = np.array(float(bm))
        out[f"rm/{i}/batch_std"] = np.array(float(bs))
        out[f"rm/{i}/mean"] = np.array(float(m.mean))
        out[f"rm/{i}/std"] = np.array(float(m.std))
        out[f"rm/{i}/var"] = np.array(float(m.var))
        out[f"rm/{i}/count"] = np.array(float(m.count))
    # Adaptive KL controller trajectory (ppo_models.py:26-44)
    kl = ppo_models.AdaptiveKLController(0.05, 6, 10000)
    currents = [0.0, 1.0, 5.9, 6.0, 7.3, 12.0, 100.0, -3.0]
    traj = []
    for c in currents:
        kl.update(c, n_steps=12)
        traj.append(kl.value)
    out["kl/currents"] = np.array(currents)
    out["kl/values"] = np.array(traj)
    fk = ppo_models.FixedKLController(0.05)
    fk.update(3.0, 12)
    out["kl/fixed"] = np.array(fk.value)
    np.savez_compressed(os.path.join(OUT, "host_state.npz"), **out)


# --------------------------------------------------------------------------- A10
def make_ilql(ilql_models, ilql_types):
    out = {}
    cfg = ilql_models.ILQLConfig(name="ilqlconfig", tau=0.7, gamma=0.99, cql_scale=0.1, awac_scale=1,
                                 alpha=0.001, steps_for_target_q_sync=5, betas=[4], two_qs=True)
    for ci, (B, L, V) in enumerate([(3, 6, 23), (2, 9, 101), (4, 5, 50257)]):
        g = gen(600 + ci)
        A = L - 1
        input_ids = torch.randint(0, V, (B, L), generator=g)
        attn = torch.ones(B, L, dtype=torch.long)
        attn[0, -2:] = 0
        actions_ixs = torch.arange(A).repeat(B, 1)
        states_ixs = torch.arange(L).repeat(B, 1)
        dones = torch.ones(B, L, dtype=torch.long)
        dones[:, -1] = 0
        if B > 2:
            dones[1, -2:] = 0
        rewards = torch.randn(B, A, generator=g)
        logits = torch.randn(B, L, V, generator=g).requires_grad_(True)
        qs = [torch.randn(B, A, V, generator=g).requires_grad_(True) for _ in range(2)]
        tqs = [torch.randn(B, A, V, generator=g) for _ in range(2)]
        vs = torch.randn(B, L, 1, generator=g).requires_grad_(True)
        batch = ilql_types.ILQLBatch(input_ids=input_ids, attention_mask=attn, rewards=rewards,
                                     states_ixs=states_ixs, actions_ixs=actions_ixs, dones=dones)
        loss, stats = cfg.loss((logits, (qs, tqs, vs)), batch)
        loss.backward()
        k = f"c{ci}"
        out[f"{k}/input_ids"] = input_ids.numpy()
        out[f"{k}/attention_mask"] = attn.numpy()
        out[f"{k}/actions_ixs"] = actions_ixs.numpy()
        out[f"{k}/states_ixs"] = states_ixs.numpy()
        out[f"{k}/dones"] = dones.numpy()
        out[f"{k}/rewards"] = rewards.numpy()
        small = V < 1000
        if small:
            out[f"{k}/logits"] = store(logits)
            for i in range(2):
                out[f"{k}/q{i}"] = store(qs[i])
                out[f"{k}/tq{i}"] = store(tqs[i])
                out[f"{k}/dq{i}"] = store(qs[i].grad)
            out[f"{k}/dlogits"] = store(logits.grad)
        else:  # wide case: regenerate inputs from the seed in the test instead of storing 10 MB
            out[f"{k}/seed"] = np.array(600 + ci)
            out[f"{k}/dlogits_sum"] = np.array(float(logits.grad.double().sum()))
            out[f"{k}/dlogits_abs_sum"] = np.array(float(logits.grad.double().abs().sum()))
            out[f"{k}/dq0_abs_sum"] = np.array(float(qs[0].grad.double().abs().sum()))
        out[f"{k}/vs"] = store(vs)
        out[f"{k}/dvs"] = store(vs.grad)
        out[f"{k}/loss"] = np.array(float(loss))
        for sk, sv in stats.items():
            out[f"{k}/stats/{sk}"] = np.array(float(sv))
    np.savez_compressed(os.path.join(OUT, "ilql_loss.npz"), **out)


# --------------------------------------------------------------------------- §8f rollout store
def load_ppo_pipeline():
    """trlx/pipeline/ppo_pipeline.py with its real package deps (trlx.data, trlx.pipeline)."""
    sys.modules.pop("trlx.data", None)
    d = _load("trlx.data", "trlx/data/__init__.py")
    d.__path__ = []
    _load("trlx.data.method_configs", "trlx/data/method_configs.py")
    types_mod = _load("trlx.data.ppo_types", "trlx/data/ppo_types.py")
    p = _load("trlx.pipeline", "trlx/pipeline/__init__.py")
    p.__path__ = []
    return _load("trlx.pipeline.ppo_pipeline", "trlx/pipeline/ppo_pipeline.py"), types_mod


def make_rollout_store(ppo_pipeline, ppo_types):
    """PPORolloutStorage.push + create_loader(shuffle=False) over three experience chunks
    of different query / response widths (the reference's own collate, ppo_pipeline.py)."""
    out = {}
    g = gen(700)
    store = ppo_pipeline.PPORolloutStorage(pad_token_id=0)
    store.clear_history()  # the reference constructs history = [None] and clears it before use
    chunks = [(3, 5, 4), (4, 7, 6), (2, 3, 2)]  # (rows, query width, response width)
    for ci, (n, wq, wr) in enumerate(chunks):
        q = torch.randint(1, 50, (n, wq), generator=g)
        q[0, :2] = 0  # the chunk's own left padding
        r = torch.randint(1, 50, (n, wr), generator=g)
        r[-1, -1] = 0
        lp, v, rw = (torch.randn(n, wr, generator=g) for _ in range(3))
        elems = [ppo_types.PPORLElement(q[i], r[i], lp[i], v[i], rw[i]) for i in range(n)]
        store.push(elems)
        for name, t in (("query", q), ("response", r), ("logprobs", lp), ("values", v), ("rewards", rw)):
            out[f"chunk{ci}/{name}"] = t.numpy()
    loader = store.create_loader(4, shuffle=False)
    for bi, batch in enumerate(loader):
        for name in ("query_tensors", "response_tensors", "logprobs", "values", "rewards"):
            out[f"batch{bi}/{name}"] = getattr(batch, name).numpy()
    out["n_batches"] = np.array(bi + 1)
    np.savez_compressed(os.path.join(OUT, "rollout_store.npz"), **out)


# --------------------------------------------------------------------------- §8f rank 3 sampling
def make_topk(ilql_models):
    """ilql_models.topk_mask (:24-28) on rows with ties at the threshold, -inf entries and
    k > V (returned unchanged)."""
    out = {}
    g = gen(800)
    xs = torch.randn(6, 37, generator=g)
    xs[1, :5] = xs[1, 5]          # a 6-way tie
    xs[2, ::3] = float("-inf")
    xs[3] = torch.round(xs[3])    # many ties
    out["xs"] = xs.numpy()
    for k in (1, 5, 20, 37, 40):
        out[f"k{k}"] = ilql_models.topk_mask(xs, k).numpy()
    np.savez_compressed(os.path.join(OUT, "topk_mask.npz"), **out)


# --------------------------------------------------------------------------- A9 model inputs
def load_ppo_model_glue():
    """trlx/model/accelerate_ppo_model.py for its module-level shift_tokens_right and the
    self-free get_model_inputs.  Its import-time base classes live in files that import ray /
    wandb / accelerate at module scope, so trlx.model and trlx.model.accelerate_base_model are
    registered as shells carrying the two names the file binds (register_model: identity
    decorator; AccelerateRLModel: an empty class) — nothing of them runs in the functions used."""
    load_ppo_pipeline()
    _load("trlx.data.configs", "trlx/data/configs.py")
    m = _shell("trlx.model")
    m.register_model = lambda c: c
    b = _shell("trlx.model.accelerate_base_model")
    b.AccelerateRLModel = type("AccelerateRLModel", (), {})
    if "trlx.model.nn.ppo_models" not in sys.modules:
        _shell("trlx.model.nn")
        _load("trlx.model.nn.ppo_models", "trlx/model/nn/ppo_models.py")
    return _load("trlx.model.accelerate_ppo_model", "trlx/model/accelerate_ppo_model.py")


def make_model_inputs(apm):
    """shift_tokens_right (:18-25) with its defaults and with explicit pad / start ids, -100
    label ids (the start id -100 too), a width-1 response; get_model_inputs (:63-76)."""
    out = {}
    g = gen(900)
    cases = {
        "plain": (torch.randint(1, 32128, (5, 9), generator=g), {}),
        "ignore": (torch.randint(-2, 50, (4, 12), generator=g), dict(pad_token_id=3, decoder_start_token_id=7)),
        "start_ignored": (torch.randint(0, 9, (3, 6), generator=g), dict(pad_token_id=5, decoder_start_token_id=-100)),
        "width1": (torch.randint(1, 100, (6, 1), generator=g), dict(decoder_start_token_id=2)),
    }
    cases["ignore"][0][cases["ignore"][0] < 0] = -100
    cases["start_ignored"][0][:, ::2] = -100
    for name, (ids, kw) in cases.items():
        out[f"{name}/ids"] = ids.numpy()
        out[f"{name}/pad"] = np.array(kw.get("pad_token_id", 0))
        out[f"{name}/start"] = np.array(kw.get("decoder_start_token_id", 0))
        out[f"{name}/out"] = apm.shift_tokens_right(ids.clone(), **kw).numpy()
    q = torch.randint(0, 32128, (4, 7), generator=g)
    r = torch.randint(0, 32128, (4, 5), generator=g)
    r[1, 3:] = -100
    a, b, c = apm.AcceleratePPOModel.get_model_inputs(None, q, r)
    out["gmi/query"], out["gmi/response"] = q.numpy(), r.numpy()
    out["gmi/input_seq"], out["gmi/labels"], out["gmi/decoder_input_ids"] = a.numpy(), b.numpy(), c.numpy()
    np.savez_compressed(os.path.join(OUT, "model_inputs.npz"), **out)


if __name__ == "__main__":
    torch.set_num_threads(4)
    only = sys.argv[1:]
    modeling, ppo_models, ilql_models, ilql_types = load_reference()
    if not only or "lsm" in only:
        make_lsm_gather(modeling)
    if not only or "kl" in only:
        make_kl_reward(modeling)
    if not only or "gae" in only:
        make_gae(ppo_models)
    if not only or "loss" in only:
        make_ppo_loss(ppo_models, modeling)
    if not only or "host" in only:
        make_host_state(modeling, ppo_models)
    if not only or "ilql" in only:
        make_ilql(ilql_models, ilql_types)
    if not only or "whiten" in only:
        make_whiten(modeling)
    if not only or "topk" in only:
        make_topk(ilql_models)
    if not only or "store" in only:
        make_rollout_store(*load_ppo_pipeline())
    if not only or "inputs" in only:
        make_model_inputs(load_ppo_model_glue())
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))
