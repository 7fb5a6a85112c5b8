"""Extractor drop-in (reference: managers/extractor.py:40-382).

Same flow and config keys: YAML config, merge of ``dirname(load_path)/
config.yaml``'s model_config, model via ``getattr(networks, config['model'])``,
detector via ``getattr(preprocess_utils, config['detector'])``, dataset via
``getattr(datasets, config['data'])``, per-image ``process`` (detect ->
denormalise -> sample+L2) and ``save_desc`` writing
``desc_root/<name>.<postfix>`` as ``np.savez(keypoints, scores, descriptors)``
(the HPatches/Aachen/ETH evaluation input format).

MI355X-specific behaviour:
* one process per GPU (torchrun / --local_rank); rank 0 broadcasts weights
  over RCCL (PoSFeat.set_parallel) and ranks extract disjoint image shards;
* descriptors are sampled from the engine's NHWC local_map (coalesced);
* no CPU path: without a gfx950 GPU the constructor raises;
* the default loop is a pipeline (``_extract_pipelined``): images are
  bucketed by size and a bucket runs as one engine batch when it holds
  ``POSFEAT_EXTRACT_GROUP`` images (default 32; at most
  ``POSFEAT_EXTRACT_HOLD`` images wait, default 4 groups; instance norm and
  eval BatchNorm are per image, so each image's maps are those of a batch-1
  run up to fp32 summation order); only the uint8 image crosses PCIe (one
  fork-excluded pinned staging buffer per group, normalised on the device by
  posfeat_normalize_rgb8, bit-identical to the host transform); one detector
  and one sampler launch per group select every image as if alone
  (posfeat_detect_each), without host synchronisation; results come back by
  async D2H copies, and the files are written by writer threads while the
  GPU works on the next group.  The decode workers are forked at
  construction, before the model exists (a later fork stalls the device work
  that follows it).  Same files, same names, same log lines;
  ``POSFEAT_EXTRACT_PIPELINE=0`` runs the reference's serial loop;
* ``POSFEAT_EXTRACT_TIMING=1`` (serial loop) synchronises the device at the stage
  boundaries and reports per-stage time (load = decode + normalise in the
  loader, h2d, engine, detect = detector + descriptor sampler, save = D2H +
  np.savez / h5) in ``self.stats`` and the log; without it only the wall time
  and images/s are recorded (no extra synchronisation).
``save_h5`` writes the reference's layout (extractor.py:273-314:
``<desc_root>h5/<seq>/{keypoints,descriptors,scores,scales}.h5`` keyed by image
name, plus ``feat.h5`` groups for hloc) through h5py; h5py is not part of this
image, so the option fails at construction when it is missing.
Out of scope (diagnostics): save_imgs visualisation.
"""
import copy
import ctypes
import functools
import logging
import mmap
import os
import time
from collections import deque
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch
import torch.distributed as dist
import yaml

from .. import datasets, networks, ops, weights
from ..losses import preprocess_utils as putils
from ..losses.preprocess_utils import denormalize_coords, normalize_coords, sample_feat_by_coord


def _staging_buffer(n):
    """A pinned uint8 host buffer of ``n`` bytes marked MADV_DONTFORK.

    The loader's decode workers are forked from this process; a pinned page
    that is shared copy-on-write with a child is copied on the parent's next
    write, and the device's view of the buffer is then rebuilt on the next
    host-to-device copy: the first group of every extraction run took 0.2-3.2 s
    to upload 29 MB (r11i: 477 ms cold, 3242 ms in a second pass) against
    0.6 ms with the same buffers and no workers (r11j).  No worker ever reads
    the staging buffers, so they are left out of the children altogether.
    The caching host allocator hands out whole hipHostMalloc blocks (page
    aligned); the advice covers the pages inside the tensor."""
    buf = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    lo, hi = _page_range(buf)
    if hi > lo and _libc().madvise(ctypes.c_void_p(lo), ctypes.c_size_t(hi - lo),
                                   _MADV_DONTFORK) != 0:
        raise OSError(ctypes.get_errno(), "madvise(MADV_DONTFORK) on the staging buffer")
    return buf


_MADV_DONTFORK = 10   # <sys/mman.h>, Linux
_MADV_DOFORK = 11


def _page_range(buf):
    page = mmap.PAGESIZE
    a, n = buf.data_ptr(), buf.numel()
    return (a + page - 1) // page * page, (a + n) // page * page


def _release_staging_buffer(buf):
    """Undo _staging_buffer's MADV_DONTFORK before the buffer returns to torch's
    caching host allocator, whose next user may rely on fork inheriting it."""
    lo, hi = _page_range(buf)
    if hi > lo:
        _libc().madvise(ctypes.c_void_p(lo), ctypes.c_size_t(hi - lo), _MADV_DOFORK)


@functools.lru_cache(None)
def _libc():
    libc = ctypes.CDLL(None, use_errno=True)
    libc.madvise.argtypes = (ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int)
    return libc


class _StagedReader:
    """Reads each planned batch's images straight into a pinned staging buffer
    with a thread pool (the file reads release the GIL), ``ahead`` batches
    ahead of the one the device takes next.  ahead + 1 buffers in a ring: a
    buffer is refilled once the H2D copy that read it has finished."""

    def __init__(self, ds, groups, threads, ahead, bufs=None):
        self.ds, self.groups, self.ahead = ds, groups, ahead
        self.pool = ThreadPoolExecutor(threads)
        # [buffer, H2D event]; ``bufs``: staging buffers allocated beforehand
        # (Extractor._prewarm_host: sized for the plan's largest batch)
        bufs = list(bufs or [])[:ahead + 1]
        self.ring = [[bufs[k] if k < len(bufs) else None, None] for k in range(ahead + 1)]
        self.work = {}
        self.next = 0

    def _submit(self, gi):
        (h, w), idxs = self.groups[gi]
        shape = (len(idxs), h, w, 3)
        n = len(idxs) * h * w * 3
        slot = self.ring[gi % len(self.ring)]
        if slot[1] is not None:
            slot[1].synchronize()   # the H2D of the batch that used this buffer is done
            slot[1] = None
        if slot[0] is None or slot[0].numel() < n:
            if slot[0] is not None:
                _release_staging_buffer(slot[0])
            slot[0] = _staging_buffer(max(n, 2 * (slot[0].numel() if slot[0] is not None else 0)))
        st = slot[0][:n].view(shape)
        arr = st.numpy()
        self.work[gi] = (st, [self.pool.submit(self.ds.read_into, i, arr[k])
                              for k, i in enumerate(idxs)])

    def get(self, gi):
        """batch gi's filled staging view (keeps the next batches reading)"""
        while self.next < min(len(self.groups), gi + self.ahead + 1):
            self._submit(self.next)
            self.next += 1
        st, futs = self.work.pop(gi)
        for f in futs:
            f.result()
        return st

    def done_h2d(self, gi, ev):
        self.ring[gi % len(self.ring)][1] = ev

    def close(self):
        for _, futs in self.work.values():
            for f in futs:
                f.cancel()
        self.pool.shutdown(wait=True)
        for slot in self.ring:
            if slot[1] is not None:
                slot[1].synchronize()
            if slot[0] is not None:
                _release_staging_buffer(slot[0])
        self.ring = []


class Extractor:
    def __init__(self, args):
        self.args = args
        # construction phases in seconds (tools/extract_e2e.py reports them)
        self.setup_marks = {}
        t_mark = [time.perf_counter()]

        def mark(name):
            now = time.perf_counter()
            self.setup_marks[name] = now - t_mark[0]
            t_mark[0] = now

        with open(self.args.config, "r") as f:
            self.config = yaml.load(f, Loader=yaml.SafeLoader)
        self.save_root = os.path.join(".", "ckpts", self.config["output_root"])
        self.logfile = os.path.join(self.save_root, "logging_file.txt")
        self.desc_root = os.path.join(self.save_root, "desc")
        self.img_root = os.path.join(self.save_root, "image")
        self.sift_kp = self.config["use_sift"]
        if self.sift_kp:
            raise NotImplementedError("use_sift: True needs OpenCV SIFT, which is out of scope")
        self.save_npz = self.config.get("save_npz", True)
        self.save_h5 = self.config.get("save_h5", False)
        if self.save_h5:
            try:
                import h5py  # noqa: F401
            except ImportError as e:
                raise ImportError("save_h5: True needs h5py, which is not installed") from e

        cfg_path = os.path.join(os.path.dirname(str(self.config["load_path"])), "config.yaml")
        if os.path.exists(cfg_path):
            with open(cfg_path, "r") as f:
                pre_conf = yaml.load(f, Loader=yaml.SafeLoader)
            self.config["model_config"].update(pre_conf["model_config"])
            if "model" in list(pre_conf.keys()):
                self.config["model"] = pre_conf["model"]
        elif self.config["model_config"].get("backbone") in (None, "None"):
            raise FileNotFoundError(cfg_path)

        mark("config")
        self.set_device()
        mark("device")
        self.detector = getattr(putils, self.config["detector"])
        dataset = getattr(datasets, self.config["data"])
        extract_dataset = dataset(configs=self.config["data_config_extract"])
        sampler = (datasets.ShardSampler(len(extract_dataset), self.rank, self.world)
                   if self.multi_gpu else None)
        self.extract_loader = torch.utils.data.DataLoader(
            extract_dataset, batch_size=self.config["data_config_extract"]["batch_size"],
            shuffle=False, num_workers=self.config["data_config_extract"].get("workers", 0),
            collate_fn=self.my_collate, sampler=sampler, pin_memory=True)
        # The pipelined loop's decode workers are forked HERE, before the model
        # and the engine workspace exist: a fork stalls this process's next
        # device work for a time that grows with what the process has mapped
        # on the device (r11i-r11l: the first upload after a fork took 236 ms
        # in a fresh process, 3.2 s with a 25 GB engine workspace resident,
        # 0.6 ms with no fork or with the workers forked at this point)
        self._staged = self._pipelined() and self._staged_ok()
        self._early_iter = (iter(self._pipelined_loader())
                            if self._pipelined() and not self._staged else None)
        if self._early_iter is not None:
            self._warm_h2d()   # async: overlaps the model construction below
        self.set_folder_and_logger()
        mark("loader")

        tmp_model = getattr(networks, self.config["model"])
        # the seeded initial weights are drawn only if the checkpoint below
        # does not replace them (weights.deferred_seed)
        with weights.deferred_seed():
            self.model = tmp_model(self.config["model_config"], self.device)
        if self.multi_gpu:
            self.model.set_parallel(self.local_rank)
        mark("model_build")
        self.model.load_checkpoint(self.config["load_path"])
        self.model.set_eval()
        mark("checkpoint")
        self.model.engine()   # weight packing (~120 ms) belongs to construction
        mark("engine")
        if self._pipelined():
            # one workspace allocation for the whole stream (its batch shapes
            # from the file headers), while the workers decode the first
            # images -- not one allocation per larger size met on the way
            group, _ = self._group_hold()
            shapes = self._stream_shapes(group)
            if shapes:
                self.model.engine().reserve(shapes)
                mark("reserve")
                if self._staged:
                    self._prewarm_host(group)
                    mark("prewarm_host")
            elif self._staged:   # sizes unknown: the loader path after all
                self._staged = False
                self._early_iter = iter(self._pipelined_loader())
                self._warm_h2d()

        self.logger.info("use {} to detect keypoints".format(self.config["detector"]))
        if os.environ.get("POSFEAT_EXTRACT_TRACE", "0") == "1":
            t = time.perf_counter()
            torch.cuda.synchronize(self.device)
            print("[extract] construction's device work drained in %.1f ms" % (
                1e3 * (time.perf_counter() - t)), flush=True)

    def my_collate(self, batch):
        batch = list(filter(lambda b: b is not None, batch))
        return torch.utils.data.dataloader.default_collate(batch)

    def set_device(self):
        if not torch.cuda.is_available():
            raise RuntimeError("posfeat_amd Extractor needs a gfx950 GPU (no CPU path)")
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        lr = int(os.environ.get("LOCAL_RANK", getattr(self.args, "local_rank", -1)))
        self.local_rank = max(lr, 0)
        if self.world > 1:
            torch.cuda.set_device(self.local_rank)
            self.device = torch.device("cuda", self.local_rank)
            if not dist.is_initialized():
                # RCCL; POSFEAT_DIST_BACKEND=gloo: ranks sharing one device (tests)
                from ..parallel import dist_backend
                dist.init_process_group(backend=dist_backend())
            self.multi_gpu = True
            self.output_flag = self.rank == 0
        else:
            self.device = torch.device("cuda", torch.cuda.current_device())
            self.multi_gpu = False
            self.output_flag = True

    def set_folder_and_logger(self):
        if self.output_flag:
            os.makedirs(self.save_root, exist_ok=True)
            with open(os.path.join(self.save_root, "config.yaml"), "w") as fout:
                yaml.dump(self.config, fout)
            open(self.logfile, "a").close()
            os.makedirs(self.desc_root, exist_ok=True)
            os.makedirs(self.img_root, exist_ok=True)
        if self.multi_gpu:
            dist.barrier()
        self.logger = logging.getLogger("posfeat_amd.extractor")
        self.logger.setLevel(logging.INFO if self.output_flag else logging.ERROR)
        if not self.logger.handlers:
            fmt = logging.Formatter("%(asctime)s - gpu {} - %(levelname)s: %(message)s"
                                    .format(self.local_rank))
            fh = logging.FileHandler(self.logfile, mode="a")
            fh.setFormatter(fmt)
            self.logger.addHandler(fh)

    def save_desc(self, inputs, outputs, processed):
        kpt = processed["kpt"]
        feat_f = processed["desc"]
        kp_score = processed["kp_score"]
        name = inputs["name1"][0]
        save_path = os.path.join(self.desc_root, name)
        os.makedirs(os.path.dirname(save_path), exist_ok=True)
        message = "\nkpts: {}".format(kpt.shape[0])
        desc = feat_f.squeeze(0).detach().cpu().numpy()
        scores = kp_score.squeeze(0).detach().cpu().numpy()
        if self.save_npz:
            with open(save_path + ".{}".format(self.config["postfix"]), "wb") as output_file:
                np.savez(output_file, keypoints=kpt, scores=scores, descriptors=desc)
        if self.save_h5:
            h, w = inputs["im1"].shape[-2:]
            self._write_h5(name, kpt, desc, scores, w, h)
        return message

    def _write_h5(self, name, kpt, desc, scores, w, h):
        """The reference's h5 layout (extractor.py:273-314): per sequence
        keypoints/descriptors/scores/scales.h5 datasets named by the image's
        base name, and feat.h5 groups (hloc input) named by the full name."""
        import h5py
        h5_path = self.desc_root + "h5"          # the reference's path concatenation
        h5_name = name.split(".")[0]
        h5_seq = "/".join(h5_name.split("/")[:-1])
        h5_name = h5_name.split("/")[-1]
        seq_dir = os.path.join(h5_path, h5_seq)
        os.makedirs(seq_dir, exist_ok=True)
        for fname, data in (("keypoints", kpt), ("descriptors", desc), ("scores", scores),
                            ("scales", np.ones_like(scores))):
            with h5py.File(os.path.join(seq_dir, fname + ".h5"), "a") as f:
                f[h5_name] = data
        with h5py.File(os.path.join(h5_path, "feat.h5"), "a") as f:
            grp = f.create_group(name)
            grp.create_dataset("keypoints", data=kpt)
            grp.create_dataset("scores", data=scores)
            grp.create_dataset("descriptors", data=desc)
            grp.create_dataset("image_size", data=np.array([w, h]))

    def process(self, inputs, outputs, remove_pad=False):
        desc_f = outputs["local_map"]
        name = inputs["name1"][0]
        nhwc = getattr(outputs, "local_map_nhwc", None)
        if remove_pad:
            b, c, h, w = inputs["im1_ori"].shape
            pad = inputs["pad1"]
            desc_f = desc_f[:, :, :-(pad[3] // 4), :-(pad[0] // 4)]
            outputs["local_point"] = outputs["local_point"][:, :, :-(pad[3] // 4), :-(pad[0] // 4)]
            nhwc = None
        else:
            b, c, h, w = inputs["im1"].shape
        if self.config["data"] == "Aachen_Day_Night" and name.split("/")[0] == "query":
            det_cfg = self.config["detector_config_query"]
        else:
            det_cfg = self.config["detector_config"]
        coord_n, kp_score = self.detector(outputs["local_point"], **det_cfg)
        coords = denormalize_coords(coord_n, h, w)
        feat_f = sample_feat_by_coord(desc_f, coord_n, self.config["loss_distance"] == "cos",
                                      nhwc=nhwc)
        kpt = coords.cpu().numpy().squeeze(0)
        if "scale" in list(inputs.keys()):
            kpt = kpt * inputs["scale"].cpu().numpy()
        return {"kpt": kpt, "desc": feat_f, "kp_score": kp_score}

    def _pipelined(self):
        return not (os.environ.get("POSFEAT_EXTRACT_PIPELINE", "1") == "0"
                    or os.environ.get("POSFEAT_EXTRACT_TIMING", "0") == "1"
                    or self.detector is not putils.generate_kpts_single)

    @torch.no_grad()
    def extract(self):
        if not self._pipelined():
            return self._extract_serial()
        return self._extract_pipelined()

    # ------------------------------------------------------------ pipelined
    def _det_cfg(self, name):
        if self.config["data"] == "Aachen_Day_Night" and name.split("/")[0] == "query":
            return self.config["detector_config_query"]
        return self.config["detector_config"]

    def _launch_group(self, items):
        """Engine + detector + sampler for a list of same-size images, all
        enqueued on the current stream; returns (event, per-image host copies).
        items: (float image, uint8 image, name, scale)."""
        dev = self.device
        t0 = time.perf_counter()
        # the group's uint8 images go through this extractor's own pinned
        # staging buffer (two, alternating, excluded from fork: see
        # _staging_buffer): one host copy per image, one async H2D
        if all(it[1] is not None for it in items):
            shape = (len(items),) + tuple(items[0][1].shape)
            n = int(np.prod(shape))
            k = self._stage_next
            self._stage_next ^= 1
            buf, done = self._stage[k]
            if done is not None:
                done.synchronize()   # the H2D that last read this buffer has finished
            if buf is None or buf.numel() < n:
                if buf is not None:   # back to the shared pinned cache fork-inheritable
                    _release_staging_buffer(buf)
                buf = _staging_buffer(max(n, 2 * (buf.numel() if buf is not None else 0)))
            st = buf[:n].view(shape)
            for i, it in enumerate(items):
                st[i].copy_(it[1])
            self._acct_add("stage_s", t0)
            im, ev_copy = self._upload(st)
            self._stage[k] = (buf, ev_copy)
        else:
            im = torch.empty((len(items),) + tuple(items[0][0].shape), device=dev)
            for i, it in enumerate(items):
                im[i].copy_(it[0], non_blocking=True)
        return self._launch_device(im, [it[2] for it in items], [it[3] for it in items], t0)

    def _upload(self, st):
        """async H2D of a filled pinned staging view [g][h][w][3] uint8 and the
        on-device ImageNet normalisation (bit-identical to the host transform);
        returns (normalised [g][3][h][w] float, event after the copy).  The
        copy runs on its own stream: queued behind the compute stream's earlier
        groups, it held the staging buffer (and so the reader) until the device
        reached it; the compute stream waits on the copy's event instead."""
        cur = torch.cuda.current_stream(self.device)
        if getattr(self, "_h2d_stream", None) is None:
            self._h2d_stream = torch.cuda.Stream(self.device)
        with torch.cuda.stream(self._h2d_stream):   # u8 from the copy stream's pool
            u8 = torch.empty(tuple(st.shape), dtype=torch.uint8, device=self.device)
            u8.copy_(st, non_blocking=True)
            ev_copy = torch.cuda.Event()
            ev_copy.record(self._h2d_stream)
        cur.wait_event(ev_copy)
        u8.record_stream(cur)   # not reused by a later copy before the compute stream read it
        return ops.normalize_rgb8(u8), ev_copy

    def _launch_device(self, im, names, scales, t0):
        dev = self.device
        trace = os.environ.get("POSFEAT_EXTRACT_TRACE", "0") == "1"
        g, _, h, w = im.shape
        if trace:
            torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        eng = self.model.engine()
        t2 = time.perf_counter()
        out = eng.run(im, outputs=())
        self._acct_add("engine_s", t2)
        if trace:
            torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        nhwc = out["_local_map_nhwc"]
        norm = self.config["loss_distance"] == "cos"
        # one detect + one sample launch per run of images sharing a detector
        # config (Aachen query / db), each image selected as if alone
        runs = []
        i = 0
        while i < g:
            cfg = self._det_cfg(names[i])
            j = i + 1
            while j < g and self._det_cfg(names[j]) is cfg:
                j += 1
            coord_n, score, n_sel = putils.generate_kpts_each_async(
                out["local_point"][i:j], **cfg)
            desc = ops.sample_desc_nhwc(nhwc[i:j], coord_n, c=128, normalize=norm,
                                        n_valid=n_sel, each=True)
            runs.append((i, j, (n_sel, coord_n, desc, score)))
            i = j
        # the results' D2H on a copy stream: the copy (a blit kernel for a
        # device-to-pinned-host copy, 0.46 ms for a 6-image group's 25 MB of
        # descriptors, r14d) overlaps the next group's kernels instead of
        # running between them on the compute stream
        cur = torch.cuda.current_stream(dev)
        if getattr(self, "_d2h_stream", None) is None:
            self._d2h_stream = torch.cuda.Stream(dev)
        ev_done = torch.cuda.Event()
        ev_done.record(cur)
        self._d2h_stream.wait_event(ev_done)
        host = []
        with torch.cuda.stream(self._d2h_stream):
            for i, j, ts in runs:
                for t in ts:   # not reused by the compute stream before the copy read it
                    t.record_stream(self._d2h_stream)
                hs = tuple(t.to("cpu", non_blocking=True) for t in ts)
                for k in range(i, j):
                    host.append((names[k], scales[k], hs, k - i, w, h))
            ev = torch.cuda.Event()
            ev.record(self._d2h_stream)
        self._acct_add("detect_s", t3)
        if trace:
            torch.cuda.synchronize(dev)
            print("[extract]   upload+normalise %.1f ms, run %.1f ms, "
                  "detect/sample/D2H %.1f ms (synchronised)" % (
                      1e3 * (t1 - t0), 1e3 * (t3 - t2),
                      1e3 * (time.perf_counter() - t3)), flush=True)
        return ev, host

    def _acct_add(self, key, since):
        acct = getattr(self, "_acct", None)
        if acct is not None:
            acct[key] = acct.get(key, 0.0) + time.perf_counter() - since

    def _finish_group(self, ev, host, writer, futures):
        ev.synchronize()
        for name, scale, (n_sel, kpt, desc, score), r, w, h in host:
            kpt, desc, score = kpt[r:r + 1], desc[r:r + 1], score[r:r + 1]
            n = int(n_sel[r])   # the selected count (incl. the 128 raise)
            # denormalize_coords on the host: the same two fp32 roundings
            # (x * c, then + c) as the device path; a host->device copy of c
            # here would wait for the whole queue
            c = np.array([(w - 1) / 2.0, (h - 1) / 2.0], np.float32)
            k = kpt[0, :n].numpy() * c + c
            if scale is not None:
                k = k * scale
            processed = {"kpt": k, "desc": desc[:, :n], "kp_score": score[:, :n]}
            inputs = {"name1": [name], "im1": torch.empty(1, 3, h, w, device="meta")}
            if self.config["output_desc"]:
                futures.append(writer.submit(self._save_and_log, inputs, processed))
            else:
                self.logger.info(name)

    def _save_and_log(self, inputs, processed):
        self.logger.info(inputs["name1"][0] + self.save_desc(inputs, None, processed))

    def _pipelined_loader(self):
        """The pipelined loop's own loader over the same dataset and shard:
        items carry only the cropped uint8 image (the float normalisation runs
        on the device), ``POSFEAT_EXTRACT_LOAD_BATCH`` items per worker
        transaction (default 8) collated as a list (sizes may differ), and
        ``POSFEAT_EXTRACT_WORKERS`` decode workers (default: the config's
        ``workers``; an explicit 0 loads in this process).  Order is the
        sampler's, as the reference loop's.  The loader reads a shallow copy of
        the dataset with ``uint8_only`` set; the serial loader's is untouched."""
        ds = copy.copy(self.extract_loader.dataset)
        if hasattr(ds, "uint8_only"):
            ds.uint8_only = True
        cfg = self.config["data_config_extract"]
        workers = int(os.environ.get("POSFEAT_EXTRACT_WORKERS", cfg.get("workers", 4) or 0))
        nwriter = int(os.environ.get("POSFEAT_EXTRACT_WRITERS", "4"))
        self._nwriters = max(1, nwriter)
        lb = max(1, int(os.environ.get("POSFEAT_EXTRACT_LOAD_BATCH", "8")))
        sampler = (datasets.ShardSampler(len(ds), self.rank, self.world)
                   if self.multi_gpu else None)
        kw = dict(prefetch_factor=4, persistent_workers=False) if workers > 0 else {}
        return torch.utils.data.DataLoader(
            ds, batch_size=lb, shuffle=False, num_workers=workers, sampler=sampler,
            collate_fn=lambda b: [x for x in b if x is not None], pin_memory=False, **kw)

    @staticmethod
    def _plan_groups(order, sizes, group, hold):
        """The pipelined loop's batches, planned from the header sizes: images
        bucketed by size in stream order, a bucket launched when it holds
        ``group`` images, the fullest one early once ``hold`` images wait, the
        rest at the end -- the decisions the loader-driven loop takes as the
        images arrive.  Returns [((h, w), [item indices])] and the most images
        held at once."""
        groups, buckets, held, max_held = [], {}, 0, 0
        for i in order:
            key = sizes[i]
            b = buckets.setdefault(key, [])
            b.append(i)
            held += 1
            max_held = max(max_held, held)
            if len(b) >= group:
                groups.append((key, b))
                buckets[key] = []
                held -= len(b)
            elif held >= hold:
                key = max(buckets, key=lambda k: len(buckets[k]))
                held -= len(buckets[key])
                groups.append((key, buckets.pop(key)))
        for key in list(buckets):
            if buckets[key]:
                groups.append((key, buckets.pop(key)))
        return groups, max_held

    def _extract_pipelined(self):
        """Images are grouped BY SHAPE across the whole stream (one bucket per
        size, a bucket runs as one engine batch when it holds
        ``POSFEAT_EXTRACT_GROUP`` images, default 32 -- the bench batch -- and
        the remaining buckets at the end): output files are per image, so the
        processing order is free; name_list.txt keeps the loader order.
        Datasets with many image sizes (HPatches crops every image to /16,
        Aachen/ETH keep full resolution) would otherwise hold most of the
        stream in partial buckets: once ``POSFEAT_EXTRACT_HOLD`` images
        (default 4 groups) wait, the fullest bucket launches early."""
        group, hold = self._group_hold()
        if self._staged:
            return self._extract_staged_run(group, hold)
        return self._extract_pipelined_run(group, hold)

    def _group_hold(self):
        group = max(1, int(os.environ.get("POSFEAT_EXTRACT_GROUP", "32")))
        hold = max(group, int(os.environ.get("POSFEAT_EXTRACT_HOLD", str(4 * group))))
        return group, hold

    def _prewarm_host(self, group):
        """Pinned host memory for the staged run, allocated at construction
        (with the engine's workspace reserve) instead of on the way: the
        reader's ring at the plan's largest batch, and the caching host
        allocator's blocks for each batch's result copies (two per batch
        shape, freed here and reused by the run's D2H).  A pinned allocation
        is a ~8 ms hipHostMalloc of tens of MB that the launching thread waits
        for: in the HPatches-size stream nine of them sat in the first groups,
        the device idle meanwhile (r14d)."""
        _, hold = self._group_hold()
        groups, _ = self._plan_groups(self._order, self._sizes, group, hold)
        if not groups:
            return
        ahead = max(1, int(os.environ.get("POSFEAT_EXTRACT_AHEAD", "2")))
        nmax = max(len(idxs) * h * w * 3 for (h, w), idxs in groups)
        self._ring_bufs = [_staging_buffer(nmax) for _ in range(ahead + 1)]
        cfg = self.config["detector_config"]
        npts = cfg.get("num_pts", False)
        shapes = set()
        for (h, w), idxs in groups:
            P = (h - 2) * (w - 2)
            cap = min(max(int(npts), 128), P) if npts else P
            shapes.add((len(idxs), cap))
        warm = []
        for g, cap in sorted(shapes)[-4:]:   # the largest few (bounded pinned memory)
            for _ in range(2):
                warm += [torch.empty(g, dtype=torch.int32, pin_memory=True),
                         torch.empty(g, cap, 2, pin_memory=True),
                         torch.empty(g, cap, 128, pin_memory=True),
                         torch.empty(g, cap, 1, pin_memory=True)]
        del warm   # back to the caching host allocator, same size classes as the D2H

    def _extract_staged_run(self, group, hold):
        """The pipelined loop fed by the staged reader: the batches are planned
        from the file headers (_plan_groups: the same grouping as the
        loader-driven loop), and a thread pool decodes each planned batch's
        images straight into a pinned staging buffer (datasets' read_into: a
        binary PPM's rows are read into place), ``POSFEAT_EXTRACT_AHEAD``
        batches (default 2) ahead of the device.  No decode processes, no
        inter-process copy of the images, no host copy into the staging
        buffer: the host work per batch is the reads, one H2D and the launches."""
        inflight = self._inflight
        ds = self.extract_loader.dataset
        groups, max_held = self._plan_groups(self._order, self._sizes, group, hold)
        threads = max(1, int(os.environ.get("POSFEAT_EXTRACT_READERS", "8")))
        ahead = max(1, int(os.environ.get("POSFEAT_EXTRACT_AHEAD", "2")))
        reader = _StagedReader(ds, groups, threads, ahead, getattr(self, "_ring_bufs", None))
        self._ring_bufs = None   # released by the reader's close
        writer = ThreadPoolExecutor(1 if self.save_h5 else getattr(self, "_nwriters", 4))
        futures, pending = [], deque()
        self.group_shapes = []
        marks, launched = [], 0
        acct = {"loader_s": 0.0, "launch_s": 0.0, "device_wait_s": 0.0, "finish_s": 0.0}
        self._acct = acct
        t0 = time.perf_counter()
        trace = os.environ.get("POSFEAT_EXTRACT_TRACE", "0") == "1"

        def finish(p):
            tw = time.perf_counter()
            p[0].synchronize()
            tf = time.perf_counter()
            acct["device_wait_s"] += tf - tw
            self._finish_group(*p, writer, futures)
            acct["finish_s"] += time.perf_counter() - tf

        try:
            for gi, ((h, w), idxs) in enumerate(groups):
                tl = time.perf_counter()
                st = reader.get(gi)
                ta = time.perf_counter()
                acct["loader_s"] += ta - tl
                marks.append((ta - t0, launched))
                self.group_shapes.append((h, w, 3))
                im, ev_copy = self._upload(st)
                reader.done_h2d(gi, ev_copy)
                pending.append(self._launch_device(im, [ds.item_name(i) for i in idxs],
                                                   [None] * len(idxs), ta))
                launched += len(idxs)
                acct["launch_s"] += time.perf_counter() - ta
                if trace:
                    print("[extract] group %d x %s launched in %.1f ms at %.3f s" % (
                        len(idxs), (h, w, 3), 1e3 * (time.perf_counter() - ta), ta - t0),
                        flush=True)
                while len(pending) > inflight:
                    finish(pending.popleft())
            while pending:
                finish(pending.popleft())
        finally:
            reader.close()
        tw = time.perf_counter()
        for f in futures:
            f.result()
        writer.shutdown()
        acct["writer_tail_s"] = time.perf_counter() - tw
        n = len(self._order)
        self._write_name_list([(i, ds.item_name(i)) for i in self._order])
        dt = time.perf_counter() - t0
        self.stats = {"images": n, "seconds": dt, "images_per_s": n / dt if dt > 0 else 0.0,
                      "stage_ms_per_image": None, "pipeline": True, "reader": "staged",
                      "group": group, "group_marks": marks, "max_held": max_held, "hold": hold,
                      "inflight": inflight, "host": {k: round(v, 4) for k, v in acct.items()}}
        # max_held: the planned buckets' bound (the same grouping as the loader
        # loop); the reader itself holds at most ``ahead`` + 1 batches
        self.logger.info("extracted %d images in %.2fs (%.1f images/s, pipelined, staged reader, "
                         "%d groups, at most %d images held)" % (n, dt, self.stats["images_per_s"],
                                                                 len(marks), max_held))
        return n

    @property
    def _inflight(self):
        """groups enqueued on the device ahead of the one the host finishes"""
        return max(1, int(os.environ.get("POSFEAT_EXTRACT_INFLIGHT", "1")))

    def _warm_h2d(self):
        """The pinned staging buffers of ``_launch_group`` (two, alternating),
        allocated and copied to the device once here, while the model is built."""
        n = 32 * 480 * 640 * 3   # one bench-size group; buffers grow on demand
        self._stage, self._stage_next = [], 0
        for _ in range(2):
            buf = _staging_buffer(n)
            torch.empty(n, dtype=torch.uint8, device=self.device).copy_(buf, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._stage.append((buf, ev))

    def _staged_ok(self):
        """the staged reader (_extract_staged_run) serves datasets that decode
        an item into a given buffer and tell its size from the header"""
        ds = self.extract_loader.dataset
        return (os.environ.get("POSFEAT_EXTRACT_READER", "staged") != "loader"
                and hasattr(ds, "read_into") and hasattr(ds, "item_size")
                and hasattr(ds, "item_name"))

    def _stream_shapes(self, group):
        """(b, h, w) of the engine batches this stream can launch: per image
        size of the shard, batches of up to ``group`` images (from the file
        headers; None when the dataset cannot tell sizes without decoding).
        Keeps the shard's order and sizes for the staged reader."""
        ds = self.extract_loader.dataset
        if not hasattr(ds, "item_size"):
            return None
        idx = list(datasets.ShardSampler(len(ds), self.rank, self.world).idx if self.multi_gpu
                   else range(len(ds)))
        try:
            with ThreadPoolExecutor(8) as ex:
                sizes = list(ex.map(ds.item_size, idx))
        except Exception:   # unreadable header: the loader reports the file
            return None
        self._order, self._sizes = idx, dict(zip(idx, sizes))
        count = {}
        for hw in sizes:
            count[hw] = count.get(hw, 0) + 1
        return [(min(group, c), h, w) for (h, w), c in count.items()]

    def _extract_pipelined_run(self, group, hold):
        inflight = self._inflight
        writer = ThreadPoolExecutor(1 if self.save_h5 else getattr(self, "_nwriters", 4))
        futures, pending = [], deque()
        buckets = {}
        self.group_shapes = []
        names = []   # (dataset index, name) in loader order
        n = 0
        t0 = time.perf_counter()

        trace = os.environ.get("POSFEAT_EXTRACT_TRACE", "0") == "1"

        marks = []   # (launch time, images launched so far): steady-state rate
        launched = [0]

        # host-side accounting (no extra synchronisation): time in the loader,
        # enqueueing groups, waiting for the device, post-processing results
        acct = {"loader_s": 0.0, "launch_s": 0.0, "device_wait_s": 0.0, "finish_s": 0.0}
        self._acct = acct   # launch_s split into stage_s / engine_s / detect_s (+ upload)

        def finish(p):
            tw = time.perf_counter()
            p[0].synchronize()
            tf = time.perf_counter()
            acct["device_wait_s"] += tf - tw
            self._finish_group(*p, writer, futures)
            acct["finish_s"] += time.perf_counter() - tf

        def launch(items):
            ta = time.perf_counter()
            marks.append((ta - t0, launched[0]))
            self.group_shapes.append(tuple(items[0][0].shape))
            pending.append(self._launch_group(items))
            launched[0] += len(items)
            acct["launch_s"] += time.perf_counter() - ta
            if trace:
                print("[extract] group %d x %s launched in %.1f ms at %.3f s" % (
                    len(items), tuple(items[0][0].shape), 1e3 * (time.perf_counter() - ta),
                    ta - t0), flush=True)
            while len(pending) > inflight:   # groups in flight behind the host
                finish(pending.popleft())

        held = max_held = 0
        src = self._early_iter if self._early_iter is not None else self._pipelined_loader()
        self._early_iter = None
        src = iter(src)
        nbatch = -1
        while True:
            tl = time.perf_counter()
            batch = next(src, None)
            acct["loader_s"] += time.perf_counter() - tl
            if batch is None:
                break
            nbatch += 1
            if trace and nbatch < 8:
                print("[extract] loader batch %d (%d items) at %.3f s" % (
                    nbatch, len(batch), time.perf_counter() - t0), flush=True)
            for it in batch:
                u8 = it["im1_ori"]
                item = (u8, u8, it["name1"], None)
                key = tuple(u8.shape)
                b = buckets.setdefault(key, [])
                b.append(item)
                names.append((int(it["index"]), it["name1"]))
                n += 1
                held += 1
                max_held = max(max_held, held)
                if len(b) >= group:
                    launch(b)
                    buckets[key] = []
                    held -= len(b)
                elif held >= hold:   # bounded host memory: the fullest bucket goes now
                    key = max(buckets, key=lambda k: len(buckets[k]))
                    held -= len(buckets[key])
                    launch(buckets.pop(key))
        for key in list(buckets):
            if buckets[key]:
                launch(buckets.pop(key))
        while pending:
            finish(pending.popleft())
        tw = time.perf_counter()
        for f in futures:
            f.result()
        writer.shutdown()
        acct["writer_tail_s"] = time.perf_counter() - tw
        self._write_name_list(names)
        dt = time.perf_counter() - t0
        self.stats = {"images": n, "seconds": dt, "images_per_s": n / dt if dt > 0 else 0.0,
                      "stage_ms_per_image": None, "pipeline": True, "group": group,
                      "group_marks": marks, "max_held": max_held, "hold": hold,
                      "inflight": inflight, "host": {k: round(v, 4) for k, v in acct.items()}}
        self.logger.info("extracted %d images in %.2fs (%.1f images/s, pipelined, %d groups, "
                         "at most %d images held)" % (n, dt, self.stats["images_per_s"],
                                                      len(marks), max_held))
        return n

    def _write_name_list(self, names):
        """name_list.txt = "<dataset index> <name>" per image in dataset order.
        Under N > 1 every rank's (index, name) pairs are gathered to rank 0 (the
        reference wrote rank 0's shard only)."""
        if self.multi_gpu:
            allp = [None] * self.world
            dist.all_gather_object(allp, names)
            names = sorted(p for part in allp for p in part)
        if self.output_flag:
            with open(os.path.join(self.img_root, "name_list.txt"), "w") as f:
                f.write("".join("{} {}\n".format(i, nm) for i, nm in names))

    # ------------------------------------------------------------ serial
    def _extract_serial(self):
        prof = os.environ.get("POSFEAT_EXTRACT_TIMING", "0") == "1"
        stages = dict.fromkeys(("load", "h2d", "engine", "detect", "save"), 0.0)

        def mark(stage, t):
            if prof:
                torch.cuda.synchronize(self.device)
            now = time.perf_counter()
            stages[stage] += now - t
            return now

        names = []
        # dataset index of each loader item (the sampler's order; batch 1)
        smp = self.extract_loader.sampler
        order = list(smp.idx) if isinstance(smp, datasets.ShardSampler) else None
        t0 = time.perf_counter()
        n = 0
        t = t0
        for idx, inputs in enumerate(self.extract_loader):
            t = mark("load", t)
            for key, val in inputs.items():
                if key in ("name1", "pad1"):
                    continue
                inputs[key] = val.to(self.device, non_blocking=True)
            t = mark("h2d", t)
            message = inputs["name1"][0]
            outputs = self.model.extract(inputs["im1"])
            t = mark("engine", t)
            processed = self.process(inputs, outputs)
            t = mark("detect", t)
            if self.config["output_desc"]:
                message += self.save_desc(inputs, outputs, processed)
            t = mark("save", t)
            self.logger.info(message)
            names.append((order[idx] if order is not None else idx, inputs["name1"][0]))
            n += 1
        torch.cuda.synchronize(self.device)
        self._write_name_list(names)
        dt = time.perf_counter() - t0
        self.stats = {"images": n, "seconds": dt, "images_per_s": n / dt if dt > 0 else 0.0,
                      "stage_ms_per_image": ({k: 1e3 * v / max(n, 1) for k, v in stages.items()}
                                             if prof else None), "pipeline": False}
        self.logger.info("extracted %d images in %.2fs (%.1f images/s)%s" % (
            n, dt, self.stats["images_per_s"],
            "" if not prof else " stages ms/image: " + ", ".join(
                "%s %.2f" % kv for kv in self.stats["stage_ms_per_image"].items())))
        return n


__all__ = ["Extractor", "normalize_coords", "denormalize_coords"]
