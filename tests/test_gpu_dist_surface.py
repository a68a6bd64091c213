"""The drop-in distributed surface pinned to the reference's own gloo fixtures.

tests/golden/whiten.npz holds the reference's get_global_statistics / whiten outputs run
under gloo at world sizes 1, 2 and 4 (tests/golden/make_golden.py, modeling.py:9-34).
Here the SAME calls go through trlx_t5_amd on cuda:0, one process per rank (all ranks share
the one GPU of the dev box; the exchange is the product's fp64 all-reduce), and must match:
  * mean / var / count (biased variance, one all-reduce of {Σx, Σx², n});
  * whiten and whiten(shift_mean=False) on every rank's chunk, concatenated;
  * world 1 with the group initialised: the BIASED variance (SURVEY §7 trap i,
    modeling.py:26-29 vs :18-20) — the fixture's dist1 differs from its nodist;
  * RunningMoments.update in the dist branch: the Chan merge of the global batch moments
    (modeling.py:83-104; expected values from the fixture's global mean / var / count).
Tolerances: fp32 rtol 1e-5 (the product accumulates in fp64, the reference in fp32);
bf16 inputs: the reference rounds its all-reduce buffer and the whitened output to bf16
(documented deviation: the product's statistics are fp64-accurate) -> the bf16 outputs
agree within one bf16 ulp (2^-7 relative) plus 1e-2 absolute near zero.
"""
import os

import numpy as np
import pytest
import torch

from golden_util import T

pytestmark = pytest.mark.gpu
KEYS = ("f32", "bf16", "f32_big")


def _spawn(world, xs_all):
    import torch.multiprocessing as mp
    import dist_workers
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() * 7 + world) % 250
    ps = [ctx.Process(target=dist_workers.drop_in_surface_worker, args=(r, world, port, xs_all, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.fixture(scope="module")
def xs_all(golden):
    z = golden("whiten")
    return {k: T(z[f"{k}/xs"]) for k in KEYS}


@pytest.mark.parametrize("world", [1, 2, 4])
def test_drop_in_surface_matches_reference_gloo_fixtures(world, golden, xs_all):
    z = golden("whiten")
    res = _spawn(world, xs_all)
    for k in KEYS:
        bf = k == "bf16"
        tol = dict(rtol=2 ** -7, atol=1e-2) if bf else dict(rtol=1e-5, atol=1e-6)
        g_mean, g_var, g_cnt = (float(z[f"{k}/dist{world}/{n}"]) for n in ("mean", "var", "count"))
        for r in range(world):
            got = res[r][k]
            assert got["dtype"] == str(xs_all[k].dtype)  # 0-d results in xs.dtype, like the reference
            assert got["count"] == g_cnt == xs_all[k].numel()
            assert got["mean"] == pytest.approx(g_mean, rel=tol["rtol"], abs=1e-6 if not bf else 2e-2)
            assert got["var"] == pytest.approx(g_var, rel=tol["rtol"] if not bf else 2 ** -6)
        for name in ("whiten", "whiten_noshift"):
            got = torch.cat([torch.from_numpy(res[r][k][name]) for r in range(world)])
            want = T(z[f"{k}/dist{world}/{name}"]).float()
            torch.testing.assert_close(got, want, **tol, msg=f"{k} dist{world} {name}")
        # distributed=False keeps the unbiased var_mean branch although the group is up
        got = torch.cat([torch.from_numpy(res[r][k]["whiten_local"]) for r in range(world)])
        if world == 1:
            torch.testing.assert_close(got, T(z[f"{k}/nodist_disabled"]).float(), **tol)
        # RunningMoments.update (dist branch): merge of the global biased batch moments
        x = xs_all[k].double()
        mean, var, n = x.mean().item(), x.var(unbiased=False).item(), float(x.numel())
        tot = 1e-24 + n
        e_mean = mean * n / tot
        e_var = (1.0 * 1e-24 + mean ** 2 * 1e-24 * n / tot + var * n) / tot
        e_std = (e_var * tot / (tot - 1)) ** 0.5
        for r in range(world):
            rm_mean, rm_var, rm_std, rm_cnt, bm, bs = res[r][k]["rm"]
            rel = 1e-5 if not bf else 1e-5  # the update sees the same bf16-valued inputs as fp32
            assert rm_mean == pytest.approx(e_mean, rel=rel, abs=1e-6)
            assert rm_var == pytest.approx(e_var, rel=rel)
            assert rm_std == pytest.approx(e_std, rel=rel)
            assert rm_cnt == pytest.approx(tot)
            assert bm == pytest.approx(mean, rel=rel, abs=1e-6)
            assert bs == pytest.approx((var * n / (n - 1)) ** 0.5, rel=rel)


def test_world1_group_uses_biased_variance(golden, xs_all):
    """SURVEY §7 trap (i): at world size 1 with torch.distributed initialised the reference
    whitens with the biased variance; without a group, with the unbiased one.  The fixture
    shows the two differ, and the product reproduces each branch."""
    z = golden("whiten")
    res = _spawn(1, {"f32_big": xs_all["f32_big"]})
    d1 = T(z["f32_big/dist1/whiten"])
    nd = T(z["f32_big/nodist"])
    assert float((d1 - nd).abs().max()) > 1e-4  # the trap is real in the fixture
    torch.testing.assert_close(torch.from_numpy(res[0]["f32_big"]["whiten"]), d1, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(torch.from_numpy(res[0]["f32_big"]["whiten_local"]), nd, rtol=1e-5, atol=1e-6)
