"""CPU tests of the host-side logic: dataset input contract, sharding,
config plumbing, loud failure without a GPU, and the multi-process
weight-broadcast + image-sharding protocol on gloo (world_size 2)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def test_to_input_matches_reference_transform():
    """ToTensor + Normalize(ImageNet) + crop to /16 (datasets/hpatches.py:14-17, 35-38)."""
    from posfeat_amd.datasets import to_input
    im = np.random.RandomState(0).randint(0, 256, (37, 50, 3)).astype(np.uint8)
    x, crop = to_input(im)
    assert x.shape == (3, 32, 48) and crop.shape == (32, 48, 3)
    t = torch.from_numpy(im).permute(2, 0, 1).float() / 255.0
    mean = torch.tensor([0.485, 0.456, 0.406])[:, None, None]
    std = torch.tensor([0.229, 0.224, 0.225])[:, None, None]
    ref = ((t - mean) / std)[:, :32, :48]
    assert torch.allclose(x, ref, atol=1e-6)


def test_hpatches_discovery(tmp_path):
    from PIL import Image
    from posfeat_amd.datasets import HPatch_SIFT
    for seq in ("i_ajuntament", "v_boat"):
        os.makedirs(tmp_path / seq)
        for k in (1, 2):
            Image.fromarray(np.zeros((40, 52, 3), np.uint8)).save(tmp_path / seq / ("%d.ppm" % k))
    ds = HPatch_SIFT({"data_path": str(tmp_path)})
    assert len(ds) == 4
    it = ds[3]
    assert it["name1"] == "v_boat/2.ppm" and it["im1"].shape == (3, 32, 48)
    assert it["coord1"].shape == (0, 2)


def test_shard_sampler_disjoint_cover():
    from posfeat_amd.datasets import ShardSampler
    for world in (1, 2, 3, 8):
        got = sorted(i for r in range(world) for i in ShardSampler(21, r, world))
        assert got == list(range(21))


def test_no_cpu_fallback():
    """Without a GPU the product path raises instead of running on the CPU."""
    if torch.cuda.is_available():
        pytest.skip("has a GPU")
    from posfeat_amd import ops
    with pytest.raises(RuntimeError):
        ops.detect(torch.rand(1, 1, 16, 16), 1, 128)
    from posfeat_amd.losses import preprocess_utils as pu
    with pytest.raises(RuntimeError):
        pu.sample_feat_by_coord(torch.rand(1, 8, 4, 4), torch.zeros(1, 3, 2), True)


def test_configs_have_reference_keys():
    import yaml
    for name in ("extract_hpatches", "extract_aachen", "extract_ETH", "extract_synthetic"):
        c = yaml.safe_load(open(os.path.join(ROOT, "configs", name + ".yaml")))
        for k in ("output_root", "postfix", "load_path", "loss_distance", "output_desc", "model",
                  "model_config", "data", "data_config_extract", "use_sift", "detector",
                  "detector_config"):
            assert k in c, (name, k)
        assert c["detector"] == "generate_kpts_single"


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from posfeat_amd.datasets import ShardSampler
    from posfeat_amd.parallel import broadcast_weights
    from posfeat_amd.weights import seeded_state_dicts
    # rank 0 holds the real weights, the others garbage -> broadcast fixes it
    bb, hd = seeded_state_dicts(0 if rank == 0 else 7)
    broadcast_weights([bb, hd], device="cpu")
    ref_bb, ref_hd = seeded_state_dicts(0)
    ok = all(torch.equal(bb[k], ref_bb[k]) for k in bb) and \
        all(torch.equal(hd[k], ref_hd[k]) for k in hd)
    shard = list(ShardSampler(10, rank, world))
    q.put((rank, ok, shard))
    dist.destroy_process_group()


def test_gloo_broadcast_and_shard():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(60)
    assert all(ok for _, ok, _ in res)
    assert sorted(res[0][2] + res[1][2]) == list(range(10))


def _grad_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from posfeat_amd.parallel import allreduce_head_grad
    g = torch.from_numpy(np.random.RandomState(rank).randn(1000).astype(np.float32))
    w = torch.from_numpy(np.random.RandomState(99).randn(1000).astype(np.float32))
    scale = allreduce_head_grad(g)
    w_new = w - 1e-3 * scale * g          # the posfeat_sgd update with lr * scale
    q.put((rank, scale, w_new.numpy()))
    dist.destroy_process_group()


def test_gloo_head_grad_allreduce_is_ddp_mean():
    """The training step's one all-reduce + lr/world SGD equals DDP's mean-gradient
    update and leaves every rank with identical weights (trainer.py:331-356)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 1000
    procs = [ctx.Process(target=_grad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(60)
    gs = [np.random.RandomState(r).randn(1000).astype(np.float32) for r in range(2)]
    w = np.random.RandomState(99).randn(1000).astype(np.float32)
    ref = w - 1e-3 * (gs[0] + gs[1]) / 2
    assert res[0][1] == 0.5
    np.testing.assert_array_equal(res[0][2], res[1][2])
    np.testing.assert_allclose(res[0][2], ref, rtol=1e-6, atol=1e-7)


def test_bench_launcher_spawns_world2():
    """bench.py --gpus 2 with no torchrun environment starts two worker ranks
    itself (the driver's 1/2/4/8 scaling runs); the stub workload exercises
    the launch, the gloo rendezvous and the barrier / max-over-ranks timing."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--workload", "stub", "--steps", "3", "--warmup", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 prints exactly one line
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["ranks_seen"] == 2 and rec["steps"] == 3
    assert rec["value"] > 0


def test_h5_export_layout(tmp_path, monkeypatch):
    """save_h5 writes the reference's layout (managers/extractor.py:273-314):
    <desc_root>h5/<seq>/{keypoints,descriptors,scores,scales}.h5 datasets named
    by the image's base name and feat.h5 groups named by the full name.  h5py
    is not in this image: a recording stand-in checks the calls."""
    import sys
    import types
    files = {}

    class _Group(dict):
        def create_dataset(self, k, data):
            self[k] = np.asarray(data)

    class _File(dict):
        def __init__(self, path, mode):
            super().__init__()
            assert mode == "a"
            self.path = path
            files.setdefault(path, {})

        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

        def __setitem__(self, k, v):
            files[self.path][k] = np.asarray(v)

        def create_group(self, k):
            g = files[self.path][k] = _Group()
            return g

    monkeypatch.setitem(sys.modules, "h5py", types.SimpleNamespace(File=_File))
    from posfeat_amd.managers.extractor import Extractor
    ex = Extractor.__new__(Extractor)
    ex.desc_root = str(tmp_path / "desc")
    kpt = np.arange(10, dtype=np.float32).reshape(5, 2)
    desc = np.ones((5, 128), np.float32)
    sc = np.full((5, 1), 0.5, np.float32)
    ex._write_h5("v_seq/3.ppm", kpt, desc, sc, 640, 480)
    root = str(tmp_path / "desc") + "h5"
    for f, want in (("keypoints", kpt), ("descriptors", desc), ("scores", sc),
                    ("scales", np.ones_like(sc))):
        np.testing.assert_array_equal(files[os.path.join(root, "v_seq", f + ".h5")]["3"], want)
    g = files[os.path.join(root, "feat.h5")]["v_seq/3.ppm"]
    np.testing.assert_array_equal(g["image_size"], [640, 480])
    np.testing.assert_array_equal(g["keypoints"], kpt)
    assert os.path.isdir(os.path.join(root, "v_seq"))


class _FakeGroupLib:
    """Records the SyncBN group bootstrap calls (no GPU, no RCCL)."""

    def __init__(self):
        self.created = None

    def posfeat_group_unique_id(self, addr):
        import ctypes
        ctypes.memmove(addr, bytes((7 * i + 3) % 256 for i in range(128)), 128)
        return 0

    def posfeat_group_create_rccl(self, world, rank, addr, out):
        import ctypes
        self.created = (world, rank, ctypes.string_at(addr, 128))
        out._obj.value = 1000 + rank
        return 0

    def posfeat_group_create_host(self, world, rank, fn, user, out):
        self.host = (world, rank, fn)
        out._obj.value = 2000 + rank
        return 0

    def posfeat_group_destroy(self, h):
        pass


def _syncbn_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from posfeat_amd.parallel import SyncBNGroup
    fake = _FakeGroupLib()
    g = SyncBNGroup(lib=fake, shape=(4, 96, 128), transport="rccl")
    refused = False
    try:   # unequal per-rank batches are a real case (the counts are all-reduced)
        SyncBNGroup(lib=_FakeGroupLib(), shape=(4 + rank, 96, 128), transport="rccl").close()
    except ValueError:
        refused = True
    q.put((rank, fake.created, g.handle.value, refused))
    g.close()
    dist.destroy_process_group()


def test_gloo_syncbn_group_bootstrap_world2():
    """SyncBatchNorm group bootstrap (parallel.SyncBNGroup): rank 0's RCCL
    unique id reaches every rank through one broadcast over the process group
    (gloo here, RCCL on the GPU box) and each rank creates its communicator
    with (world, its rank, that id).  The cross-rank statistics themselves are
    checked on the GPU (test_gpu_syncbn.py)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 1000
    procs = [ctx.Process(target=_syncbn_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(60)
    want = bytes((7 * i + 3) % 256 for i in range(128))
    for rank, created, handle, refused in res:
        assert created == (2, rank, want)
        assert handle == 1000 + rank
        assert not refused


def _syncbn_host_worker(rank, world, port, q):
    import ctypes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from posfeat_amd.parallel import SyncBNGroup
    fake = _FakeGroupLib()
    g = SyncBNGroup(lib=fake)            # a gloo group: the host transport
    w, r, fn = fake.host
    # the C side's call: n doubles in a host buffer, summed in place over ranks
    buf = (ctypes.c_double * 5)(*[rank + 0.5 * i for i in range(5)])
    rc = ctypes.cast(fn, SyncBNGroup._HostFn)(buf, 5, None)
    q.put((rank, g.transport, w, r, g.handle.value, rc, list(buf)))
    g.close()
    dist.destroy_process_group()


def test_gloo_syncbn_host_transport_world2():
    """SyncBatchNorm over a gloo process group (parallel.SyncBNGroup host
    transport, group.hip posfeat_group_create_host): the callback the C side
    calls with a host copy of each statistics vector sums it over the ranks
    in place (dist.all_reduce).  The GPU side runs in test_gpu_multirank.py."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 1000
    procs = [ctx.Process(target=_syncbn_host_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(60)
    for rank, transport, w, r, handle, rc, buf in res:
        assert (transport, w, r, handle, rc) == ("host", 2, rank, 2000 + rank, 0)
        assert buf == [1.0 + i for i in range(5)]   # (0 + .5 i) + (1 + .5 i)


def test_extract_plan_groups_matches_loader_bucketing():
    """The staged reader's batches (Extractor._plan_groups, from the header
    sizes) are the batches the loader-driven loop forms as images arrive:
    same bucketing, group and hold rules, same order."""
    import random
    from posfeat_amd.managers.extractor import Extractor
    rnd = random.Random(3)
    for group, hold, nsizes in ((32, 128, 3), (4, 5, 6), (6, 24, 40), (1, 1, 2)):
        order = list(range(300))
        pool = [(480, 640), (592, 800), (752, 992)] + [(16 * (30 + j), 16 * (40 + j))
                                                       for j in range(nsizes)]
        sizes = {i: pool[rnd.randrange(nsizes)] for i in order}
        groups, max_held = Extractor._plan_groups(order, sizes, group, hold)
        # the loader-driven loop (_extract_pipelined_run), restated
        ref, buckets, held = [], {}, 0
        for i in order:
            key = sizes[i]
            b = buckets.setdefault(key, [])
            b.append(i)
            held += 1
            if len(b) >= group:
                ref.append((key, b))
                buckets[key] = []
                held -= len(b)
            elif held >= hold:
                k = max(buckets, key=lambda k: len(buckets[k]))
                held -= len(buckets[k])
                ref.append((k, buckets.pop(k)))
        ref += [(k, v) for k, v in buckets.items() if v]
        assert groups == ref
        assert sorted(i for _, g in groups for i in g) == order
        assert max_held <= hold


def test_dataset_read_into_matches_decode(tmp_path):
    """read_into (the staged reader's decode: binary PPM rows read in place,
    else PIL) gives exactly crop16(_read(path)), for widths that need and
    need not a crop, a header comment, and a non-PPM file."""
    import numpy as np
    from PIL import Image
    from posfeat_amd import datasets
    d = tmp_path / "seq"
    d.mkdir()
    rs = np.random.RandomState(0)
    for k, (h, w) in enumerate([(480, 640), (500, 650), (97, 33)]):
        Image.fromarray(rs.randint(0, 256, (h, w, 3)).astype(np.uint8)).save(str(d / ("%d.ppm" % k)))
    a = rs.randint(0, 256, (64, 80, 3)).astype(np.uint8)
    (d / "8.ppm").write_bytes(b"P6\n# comment\n80 64\n255\n" + a.tobytes())
    Image.fromarray(rs.randint(0, 256, (50, 70)).astype(np.uint8)).save(str(d / "9.ppm"))  # P5
    ds = datasets.HPatch_SIFT({"data_path": str(tmp_path)})
    assert len(ds) == 5
    for i in range(len(ds)):
        h, w = ds.item_size(i)
        out = np.empty((h, w, 3), np.uint8)
        ds.read_into(i, out)
        np.testing.assert_array_equal(out, datasets.crop16(datasets._read(ds.imfs[i])))
    syn = datasets.SyntheticImages({"num_images": 3, "sizes": [[40, 50], [32, 48]]})
    for i in range(3):
        h, w = syn.item_size(i)
        out = np.empty((h, w, 3), np.uint8)
        syn.read_into(i, out)
        syn.uint8_only = True
        np.testing.assert_array_equal(out, syn[i]["im1_ori"].numpy())
        assert syn.item_name(i) == syn[i]["name1"]
