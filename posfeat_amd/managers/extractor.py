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
* no CPU path: without a gfx950 GPU the constructor raises.
Out of scope (diagnostics): save_imgs visualisation, h5 export.
"""
import logging
import os
import time

import numpy as np
import torch
import torch.distributed as dist
import yaml

from .. import datasets, networks
from ..losses import preprocess_utils as putils
from ..losses.preprocess_utils import denormalize_coords, normalize_coords, sample_feat_by_coord


class Extractor:
    def __init__(self, args):
        self.args = args
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
            raise NotImplementedError("save_h5 (h5py export) is out of scope")

        cfg_path = os.path.join(os.path.dirname(str(self.config["load_path"])), "config.yaml")
        if os.path.exists(cfg_path):
            with open(cfg_path, "r") as f:
                pre_conf = yaml.load(f, Loader=yaml.SafeLoader)
            self.config["model_config"].update(pre_conf["model_config"])
            if "model" in list(pre_conf.keys()):
                self.config["model"] = pre_conf["model"]
        elif self.config["model_config"].get("backbone") in (None, "None"):
            raise FileNotFoundError(cfg_path)

        self.set_device()
        self.set_folder_and_logger()

        tmp_model = getattr(networks, self.config["model"])
        self.model = tmp_model(self.config["model_config"], self.device)
        if self.multi_gpu:
            self.model.set_parallel(self.local_rank)
        self.model.load_checkpoint(self.config["load_path"])
        self.model.set_eval()

        self.detector = getattr(putils, self.config["detector"])
        self.logger.info("use {} to detect keypoints".format(self.config["detector"]))

        dataset = getattr(datasets, self.config["data"])
        extract_dataset = dataset(configs=self.config["data_config_extract"])
        sampler = (datasets.ShardSampler(len(extract_dataset), self.rank, self.world)
                   if self.multi_gpu else None)
        self.extract_loader = torch.utils.data.DataLoader(
            extract_dataset, batch_size=self.config["data_config_extract"]["batch_size"],
            shuffle=False, num_workers=self.config["data_config_extract"].get("workers", 0),
            collate_fn=self.my_collate, sampler=sampler)

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
                dist.init_process_group(backend="nccl")
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
        if self.save_npz:
            desc = feat_f.squeeze(0).detach().cpu().numpy()
            scores = kp_score.squeeze(0).detach().cpu().numpy()
            with open(save_path + ".{}".format(self.config["postfix"]), "wb") as output_file:
                np.savez(output_file, keypoints=kpt, scores=scores, descriptors=desc)
        return message

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

    @torch.no_grad()
    def extract(self):
        name_list = ""
        t0 = time.time()
        n = 0
        for idx, inputs in enumerate(self.extract_loader):
            for key, val in inputs.items():
                if key in ("name1", "pad1"):
                    continue
                inputs[key] = val.to(self.device, non_blocking=True)
            message = inputs["name1"][0]
            outputs = self.model.extract(inputs["im1"])
            processed = self.process(inputs, outputs)
            if self.config["output_desc"]:
                message += self.save_desc(inputs, outputs, processed)
            self.logger.info(message)
            name_list += "{} {}\n".format(idx, inputs["name1"][0])
            n += 1
        if self.output_flag:
            with open(os.path.join(self.img_root, "name_list.txt"), "w") as f:
                f.write(name_list)
        dt = time.time() - t0
        self.logger.info("extracted %d images in %.2fs" % (n, dt))
        return n


__all__ = ["Extractor", "normalize_coords", "denormalize_coords"]
