"""Two ranks through the real entry points, sharing the one GPU of the box.

BASELINE configs[3] (Aachen extraction image-sharded over ranks) and configs[4]
(descriptor training under DDP + SyncBatchNorm) need 8 GPUs; what a one-GPU
box can check is that the multi-rank code paths give the world-1 results:

* ``extract.py --config configs/extract_aachen.yaml`` as two ranks (RANK /
  WORLD_SIZE / LOCAL_RANK=0 as torchrun sets them; the weights broadcast from
  rank 0, ShardSampler shards, name_list gathered to rank 0) writes, over both
  ranks, exactly the files of the world-1 run with bit-identical arrays
  (/root/reference/managers/extractor.py:95-97,109-129,318-382).  Both runs
  use POSFEAT_EXTRACT_GROUP=1 (every image its own engine batch), so the batch
  composition cannot differ between the runs.
* one descriptor-training step through the Trainer's plug points
  (PoSFeat.set_parallel + forward + loss.backward(), tests/mr_worker.py;
  /root/reference/managers/trainer.py:128-173,293-331) as two ranks with half
  the batch each: SyncBatchNorm statistics over the ranks (the host transport
  of parallel.SyncBNGroup: gloo between the processes) and DDP's gradient
  mean.  On the golden fixture case the world-2 gradient meets the fp64
  fixture bound of test_bb_train; at the bench shape (8 pairs at 480x640)
  each rank's maps equal its rows of the world-1 run, the running statistics
  the world-1 update, and the mean gradient the world-1 gradient within
  test_gpu_syncbn's two-summation-order bound.

The subprocesses start before any GPU call of their own and join a gloo
process group (POSFEAT_DIST_BACKEND=gloo): RCCL refuses two ranks on one
device.  The RCCL path itself runs in the driver's 8-GPU bench.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import yaml

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _launch(argv, world, cwd, env_extra=None, timeout=600):
    """Start ``world`` ranks of argv (torchrun's environment contract, all on
    device 0, gloo), wait for all; a failing rank takes the others down."""
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0",
                   LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   POSFEAT_DIST_BACKEND="gloo", **(env_extra or {}))
        env["PYTHONPATH"] = os.pathsep.join([ROOT, HERE, env.get("PYTHONPATH", "")])
        procs.append(subprocess.Popen([sys.executable] + argv, cwd=str(cwd), env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, "rank %d failed:\n%s" % (r, o[-4000:])
    return outs


# ---- configs[3]: Aachen extraction, image-sharded --------------------------

def _aachen_tree(root):
    from PIL import Image
    rs = np.random.RandomState(11)
    for sub, n, hw in (("db", 3, (128, 160)), ("db", 2, (160, 192)),
                       (os.path.join("query", "day", "nexus5x"), 2, (128, 160)),
                       (os.path.join("query", "night", "nexus5x"), 2, (160, 192))):
        d = os.path.join(root, sub)
        os.makedirs(d, exist_ok=True)
        for i in range(n):
            im = rs.randint(0, 256, (hw[0] // 8, hw[1] // 8, 3)).astype(np.uint8)
            im = Image.fromarray(im).resize((hw[1], hw[0]), Image.BILINEAR)
            im.save(os.path.join(d, "%dx%d_%d.jpg" % (hw[0], hw[1], i)), quality=95)


def _files(desc):
    out = {}
    for dp, _, fs in os.walk(desc):
        for f in fs:
            out[os.path.relpath(os.path.join(dp, f), desc)] = os.path.join(dp, f)
    return out


def test_extract_aachen_two_ranks_match_one_rank(gpu, tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import extract_e2e
    data = tmp_path / "aachen"
    _aachen_tree(str(data))
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "extract_aachen.yaml")))
    cfg["data_config_extract"]["data_path"] = str(data)
    cfg["detector_config_query"].update(nms_radius=1, thr=0.1, num_pts=150)
    env = {"POSFEAT_EXTRACT_GROUP": "1"}
    roots = {}
    for world in (1, 2):
        cwd = tmp_path / ("w%d" % world)
        cwd.mkdir()
        extract_e2e.make_checkpoint(str(cwd))     # load_path is relative to the cwd
        if world == 1:
            from test_gpu_extract import run_extract
            roots[world] = run_extract(cfg, cwd, env=env)
        else:
            p = str(cwd / "cfg.yaml")
            yaml.safe_dump(cfg, open(p, "w"))
            _launch([os.path.join(ROOT, "extract.py"), "--config", p], 2, cwd, env)
            roots[world] = os.path.join(str(cwd), "ckpts", cfg["output_root"])
    f1, f2 = _files(os.path.join(roots[1], "desc")), _files(os.path.join(roots[2], "desc"))
    assert len(f1) == 9 and sorted(f1) == sorted(f2), (sorted(f1), sorted(f2))
    for name in sorted(f1):
        a, b = np.load(f1[name]), np.load(f2[name])
        assert sorted(a.files) == sorted(b.files) == ["descriptors", "keypoints", "scores"]
        for k in a.files:
            assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape, (name, k)
            assert a[k].tobytes() == b[k].tobytes(), "%s/%s differs between world 1 and 2" % (
                name, k)
    n1 = open(os.path.join(roots[1], "image", "name_list.txt")).read()
    n2 = open(os.path.join(roots[2], "image", "name_list.txt")).read()
    assert n1 == n2 and len(n1.splitlines()) == 9


# ---- configs[4] / configs[2]: descriptor training under DDP + SyncBN -------

def _train(tmp_path, case, world):
    """Run tests/mr_worker.py as ``world`` ranks; returns each rank's npz."""
    out = str(tmp_path / ("%s_w%d_r{rank}.npz" % (case, world)))
    _launch([os.path.join(HERE, "mr_worker.py"), case, out], world, tmp_path)
    res = []
    for r in range(world):
        d = np.load(out.format(rank=r))
        res.append({k: d[k] for k in d.files})
    return res


def test_train_desc_two_ranks_syncbn_fixture_bound(gpu, tmp_path):
    """Fixture case (tests/golden/bb_grad.npz, 2 pairs at 128x160): one pair per
    rank; world x the DDP mean gradient is the summed-loss gradient the fp64
    fixture holds, and it meets test_bb_train's per-tensor bound."""
    from test_bb_train import _check_grads64
    d = np.load(os.path.join(GOLDEN, "bb_grad.npz"))
    ranks = _train(tmp_path, "fixture", 2)
    for k in ranks[0]:
        if k.startswith("g/") or k.startswith("s/"):   # DDP: every rank holds the same
            np.testing.assert_array_equal(ranks[0][k], ranks[1][k], err_msg=k)
    got = {k[2:]: 2.0 * v for k, v in ranks[0].items() if k.startswith("g/")}
    _check_grads64(got, d)


def test_train_desc_two_ranks_syncbn_bench_shape(gpu, tmp_path):
    """configs[2]'s bench shape (8 pairs at 480x640): world 2 x 4 pairs against
    world 1 x 8 pairs."""
    one = _train(tmp_path, "bench", 1)[0]
    ranks = _train(tmp_path, "bench", 2)
    b = one["lm1"].shape[0] // 2
    for r, res in enumerate(ranks):
        for s in ("lm1", "lm2"):
            ref = one[s][r * b:(r + 1) * b]
            bound = 1e-5 * float(np.abs(one[s]).max())   # tests/tol.py's map bound
            e = float(np.abs(res[s] - ref).max())
            print("rank %d %s: max abs err %.3e (bound %.3e)" % (r, s, e, bound))
            assert e <= bound, "rank %d %s map err %g" % (r, s, e)
        for k in one:
            if k.startswith("s/"):
                np.testing.assert_allclose(res[k], one[k], rtol=1e-5, atol=1e-6, err_msg=k)
    for k in ranks[0]:
        if k.startswith("g/"):
            np.testing.assert_array_equal(ranks[0][k], ranks[1][k], err_msg=k)
    gref = {k: v for k, v in one.items() if k.startswith("g/")}
    assert sorted(gref) == sorted(k for k in ranks[0] if k.startswith("g/"))
    floor = 1e-4 * max(float(np.abs(v).max()) for v in gref.values())
    num = den = 0.0
    for k, v in gref.items():
        g = ranks[0][k]
        e = float(np.abs(g - v).max())
        assert e <= 3e-2 * float(np.abs(v).max()) + floor, "%s: err %g of max %g" % (
            k, e, float(np.abs(v).max()))
        num += float(((g - v) ** 2).sum())
        den += float((v ** 2).sum())
    print("world 2 vs world 1: relative L2 of the gradient %.2e" % (num ** 0.5 / den ** 0.5))
    assert num ** 0.5 <= 2e-3 * den ** 0.5
