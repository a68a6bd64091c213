"""CPU-only checks of the host side: the C-ABI library's exported symbols, the ctypes
signature table, host scalar logic (KL controllers, RunningMoments merge, flatten_dict,
stats layout), grad-buffer phase logic, and the gloo (world 2) DP statistics exchange."""
import os
import re
import subprocess

import numpy as np
import pytest
import torch

import trlx_t5_amd as P
from trlx_t5_amd import _lib
from trlx_t5_amd.modeling import _allreduce_moments, merge_moments, moments_to_mean_var
from golden_util import T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "trlx_t5_amd.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(trlx_\w+)\s*\(", txt, flags=re.M)))


def test_header_declares_the_binding_table():
    assert set(header_functions()) == set(_lib.SIGNATURES)


@pytest.fixture(scope="module")
def built_lib():
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "trlx-t5_amd", "csrc"), "-j8"])
    return _lib.load()


def test_library_exports_every_declared_symbol(built_lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = set(re.findall(r"\bT (trlx_\w+)", out))
    missing = set(header_functions()) - exported
    assert not missing, f"declared but not exported: {missing}"
    assert built_lib.trlx_abi_version() == _lib.ABI_VERSION


@pytest.fixture(scope="module")
def fresh_lib(tmp_path_factory):
    """The library built from the sources at HEAD into a scratch dir (never the in-tree .so,
    which may predate the sources): a tree that does not compile fails the CPU suite."""
    d = tmp_path_factory.mktemp("fresh_build")
    out = d / "libtrlx_t5_amd.so"
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "trlx-t5_amd", "csrc"), f"-j{min(8, os.cpu_count() or 1)}",
                        f"OUT={out}", f"BUILD={d / 'obj'}"], capture_output=True, text=True)
    assert r.returncode == 0, "HIP library does not build from source:\n" + r.stderr[-4000:]
    return str(out)


def test_fresh_build_exports_exactly_the_header(fresh_lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", fresh_lib]).decode()
    exported = set(re.findall(r"\bT (trlx_\w+)", out))
    declared = set(header_functions())
    assert declared - exported == set(), f"declared but not exported: {declared - exported}"
    assert exported - declared == set(), f"exported but not declared / bound: {exported - declared}"
    assert b"gfx950" in open(fresh_lib, "rb").read()
    in_tree = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode() \
        if os.path.exists(_lib.LIB_PATH) else ""
    assert set(re.findall(r"\bT (trlx_\w+)", in_tree)) == exported, "in-tree .so is stale: rebuild with make"


def test_capi_consumer_builds_against_the_fresh_library(fresh_lib, tmp_path):
    """tests/capi/capi_check.cpp (a C++ caller of the C ABI, no torch) compiles and links
    against the library built from HEAD's sources."""
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "capi"), f"OUT={tmp_path / 'capi_check'}",
                        f"LIBDIR={os.path.dirname(fresh_lib)}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    assert os.path.exists(tmp_path / "capi_check")


def test_library_is_gfx950_code(built_lib):
    assert b"gfx950" in open(_lib.LIB_PATH, "rb").read()


def test_kernels_refuse_cpu_tensors():
    x = torch.randn(2, 3, 11)
    y = torch.zeros(2, 3, dtype=torch.long)
    with pytest.raises(ValueError, match="ROCm"):
        P.logprobs_from_logits(x, y)
    with pytest.raises(ValueError):
        P.whiten(torch.randn(4, 4))


def test_kl_controllers(golden):
    z = golden("host_state")
    kl = P.AdaptiveKLController(0.05, 6, 10000)
    for c, want in zip(z["kl/currents"], z["kl/values"]):
        kl.update(float(c), n_steps=12)
        assert kl.value == pytest.approx(float(want), rel=1e-15)
    fk = P.FixedKLController(0.05)
    fk.update(3.0, 12)
    assert fk.value == float(z["kl/fixed"])


def test_running_moments_merge_kat(golden):
    """The reference KAT (tests/test_ppo.py:49-66) through the host merge the device path uses."""
    z = golden("host_state")
    mean, var, count = 0.0, 1.0, 1e-24
    for i in range(4):
        a = np.asarray(z[f"rm/{i}/in"], dtype=np.float64)
        n = a.size
        xm, xv = a.mean(), a.var()
        mean, var, std, count = merge_moments(mean, var, count, xm, xv, n)
        assert mean == pytest.approx(float(z[f"rm/{i}/mean"]), rel=1e-12)
        assert std == pytest.approx(float(z[f"rm/{i}/std"]), rel=1e-12)
        assert (xv * n / (n - 1)) ** 0.5 == pytest.approx(float(z[f"rm/{i}/batch_std"]), rel=1e-12)
    allv = np.concatenate([np.asarray(z[f"rm/{i}/in"]) for i in range(4)])
    assert mean == pytest.approx(allv.mean(), abs=1e-6)
    assert std == pytest.approx(allv.std(ddof=1), abs=1e-6)


def test_flatten_dict_and_stats_layout():
    d = {"losses": {"a": 1, "b": {"c": 2}}, "ratio": 3}
    assert P.flatten_dict(d) == {"losses/a": 1, "losses/b/c": 2, "ratio": 3}
    assert len(P.STATS_KEYS) == _lib.PPO_STATS
    from oracle import ppo_oracle as orc
    n = 6
    _, stats = orc.ppo_loss(torch.zeros(2, 3), torch.zeros(2, 3), torch.zeros(2, 3), torch.zeros(2, 3),
                            torch.zeros(2, 3), torch.ones(2, 3), torch.ones(2, 3, dtype=torch.long))
    assert set(stats) == set(P.STATS_KEYS)
    del n


@pytest.mark.parametrize("shape_stride", [((3, 5, 37), None), ((4, 6, 11), "slice")])
def test_grad_buffer_phase(shape_stride):
    shape, kind = shape_stride
    full = torch.randn(shape[0] + 1, *shape[1:], dtype=torch.bfloat16)
    x = full[:, :-1] if kind else full[:-1]
    for off in range(4):
        xv = full.view(-1)[off:off + x.numel()].view(x.shape) if kind is None else x
        d = P.grad_buffer_like(xv)
        assert d.shape == xv.shape and d.stride() == xv.stride()
        assert (d.data_ptr() - xv.data_ptr()) % 256 == 0


@pytest.mark.parametrize("world", [2])
def test_dp_whitening_statistics_gloo(golden, world):
    """world-2 gloo: the one-shot {sum, sumsq, n} all-reduce reproduces the reference's
    two-phase global mean / biased variance (modeling.py:9-21, fixture from gloo ranks)."""
    import torch.multiprocessing as mp
    z = golden("whiten")
    xs = T(z["f32_big/xs"])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 200
    import dist_workers
    ps = [ctx.Process(target=dist_workers.whiten_stats_worker, args=(r, world, port, xs, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    for _, mean, var, cnt in res:
        assert mean == pytest.approx(float(z[f"f32_big/dist{world}/mean"]), rel=1e-6)
        assert var == pytest.approx(float(z[f"f32_big/dist{world}/var"]), rel=1e-6)
        assert cnt == float(z[f"f32_big/dist{world}/count"])
        w = (xs - mean) * torch.rsqrt(torch.tensor(var, dtype=torch.float32) + 1e-8)
        torch.testing.assert_close(w, T(z[f"f32_big/dist{world}/whiten"]), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("cname,mirror", [("trlx_ilql_args", "IlqlArgs"), ("trlx_score_ctl", "ScoreCtl"),
                                           ("trlx_kl_ctl", "KlCtl"), ("trlx_gae_split_args", "GaeSplitArgs")])
def test_struct_layout_matches_header(tmp_path, cname, mirror):
    """The ctypes mirrors of the C-ABI POD structs have the C compiler's field offsets."""
    cls = getattr(_lib, mirror)
    fields = [f[0] for f in cls._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "trlx_t5_amd.h"\nint main(void){\n'
                   + "".join(f'printf("%zu\\n", offsetof({cname}, {f}));\n' for f in fields)
                   + f'printf("%zu\\n", sizeof({cname}));\nreturn 0;}}\n')
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = [int(v) for v in subprocess.check_output([str(exe)]).decode().split()]
    want = [getattr(cls, f).offset for f in fields] + [__import__("ctypes").sizeof(cls)]
    assert got == want


def test_ctl_slot_constants_match_header():
    txt = open(HEADER).read()
    for name in ["SLOTS", "MEAN", "VAR", "STD", "COUNT", "REF_MEAN", "REF_STD", "REF_SET", "KL_COEF", "BATCH_MEAN",
                 "BATCH_STD", "KL_UPDATES", "LAST_KL"]:
        m = re.search(rf"#define TRLX_CTL_{name} (\d+)", txt)
        assert m and int(m.group(1)) == getattr(_lib, f"CTL_{name}"), name
    for name in ["NONE", "RUNNING", "REF"]:
        m = re.search(rf"TRLX_SCALE_{name} = (\d+)", txt)
        assert m and int(m.group(1)) == getattr(_lib, f"SCALE_{name}"), name


def test_control_state_refuses_bad_scale():
    with pytest.raises(ValueError, match="scale_reward"):
        P.PPOControlState("cpu", scale_reward="bogus")


def test_ilql_refuses_cpu_tensors():
    cfg = P.ILQLConfig()
    B, L, V = 2, 4, 7
    A = L - 1
    b = P.ILQLBatch(torch.zeros(B, L, dtype=torch.long), torch.ones(B, L, dtype=torch.long), torch.zeros(B, A),
                    torch.arange(L).repeat(B, 1), torch.arange(A).repeat(B, 1), torch.ones(B, L, dtype=torch.long))
    qs = [torch.randn(B, A, V) for _ in range(2)]
    with pytest.raises(ValueError, match="ROCm"):
        cfg.loss((torch.randn(B, L, V), (qs, qs, torch.randn(B, L, 1))), b)


def test_tuning_rejects_removed_forms_and_restores():
    """The dropped loss-side forms (round-5 H-sliced engines, the 32x32 pair forward) are no
    longer selectable; _lib.tuning restores the previous knob values (host-only calls)."""
    import trlx_t5_amd as P
    L = P._lib
    for key, val in (("lmloss_fwd", 1), ("lmloss_fwd", 3), ("lmloss_fwd", 4), ("lmloss_dw", 2), ("lmloss_dw", 3)):
        with pytest.raises(ValueError):
            L.set_tuning(key, val)
    L.set_tuning("lmloss_fwd", 2)
    L.set_tuning("lmloss_fwd", 0)
    L.set_tuning("lmloss_dw", 4)
    with L.tuning(lmloss_dw=1, lmloss_splits=3):
        assert L._TUNED["lmloss_dw"] == 1 and L._TUNED["lmloss_splits"] == 3
    assert L._TUNED["lmloss_dw"] == 4 and L._TUNED["lmloss_splits"] == 0
    with pytest.raises(RuntimeError):
        with L.tuning(lmloss_dw=1):
            raise RuntimeError("inside")
    assert L._TUNED["lmloss_dw"] == 4
    L.set_tuning("lmloss_dw", 0)


def test_savep_region_sizes():
    """The saved-P region of the drop-in pair: the P tiles (⌈V/64⌉ x 2⌈N/64⌉ x 4 KB, the size of
    bf16 logits rounded to tiles) + 8 fp32 split scales per token; the PPO entries' saved-P
    workspace holds the P tiles and the per-split scaled h rows (8·N·H bf16) on top of the
    recompute plan's."""
    import trlx_t5_amd as P
    q = P._lib.query
    N, H, V = 6144, 768, 50257
    pbytes = ((V + 63) // 64) * 2 * ((N + 63) // 64) * 4096
    assert q("trlx_lmhead_savep_bytes", N, H, V) == pbytes + 8 * N * 4
    assert pbytes >= 2 * N * V
    big, small = q("trlx_ppo_loss_from_hidden_workspace_bytes", N, H, V), q("trlx_lmhead_loss_workspace_bytes", N, H, V)
    assert big - small >= pbytes + 8 * N * H * 2
    assert q("trlx_ppo_loss_from_hidden_plan", N, H, V, big) == 1
    assert q("trlx_ppo_loss_from_hidden_plan", N, H, V, small) == 0


def test_hot_path_refuses_bad_loss_norm():
    import trlx_t5_amd as P
    with pytest.raises(ValueError):
        P.PPOHotPath(P.PPOConfig(), 2, 3, 5, torch.bfloat16, "cpu", kl_coef=0.05, loss_norm="batch")


@pytest.mark.parametrize("n", [2, 4])
def test_bench_launcher_spawns_ranks(n):
    """`bench.py --gpus N` with no WORLD_SIZE starts N ranks itself (never a silent 1-rank
    run); the dry run joins them in a gloo group and rank 0 prints one line with n_gpus N."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([__import__("sys").executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run"],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    rec = __import__("json").loads(lines[0])
    assert rec["n_gpus"] == n and rec["ok"] and sorted(map(tuple, rec["ranks"])) == [(i, i) for i in range(n)]


def _bench_env():
    return {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}


def test_bench_launcher_reports_rank_fields():
    """The line carries the communicator's rank count and the per-rank step-time spread;
    C3 at N > 1 defaults to BASELINE's global batch 512 (strong scaling)."""
    import json
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--config", "c3", "--dry-run"],
                       capture_output=True, text=True, env=_bench_env(), timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert rec["config"]["global_batch"] == 512 and rec["config"]["rows_per_gpu"] == 128
    assert rec["config"]["scaling"] == "strong" and rec["config"]["comm_nranks"] == 4
    rs = rec["rank_ms_per_step"]
    assert rs["ranks"] == 4 and 0 < rs["min"] < rs["max"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "c2", "--dry-run"],
                       capture_output=True, text=True, env=_bench_env(), timeout=240)
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert rec["config"]["global_batch"] == 256 and rec["config"]["scaling"] == "weak"


def test_bench_launcher_deadline_stops_a_stuck_rank():
    """A rank that never exits (and ignores SIGTERM) no longer holds the launcher: after
    --rank-timeout every live rank is stopped (SIGTERM, then SIGKILL), the stuck ranks are
    named on stderr and the launcher exits non-zero."""
    import sys
    import time
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                        "--dry-run-hang-rank", "1", "--rank-timeout", "8"],
                       capture_output=True, text=True, env=_bench_env(), timeout=120)
    took = time.monotonic() - t0
    assert r.returncode == 124, (r.returncode, r.stderr[-2000:])
    assert "had not exited" in r.stderr and "1]" in r.stderr and "killed" in r.stderr
    assert took < 60


def test_bench_refuses_mislabelled_world():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([__import__("sys").executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--dry-run"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
