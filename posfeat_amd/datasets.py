"""Extraction datasets with the reference's file discovery and input contract.

Reference: datasets/hpatches.py:8-46, datasets/aachen.py:10-64,
datasets/ETH_local_feature.py:10-59.  Each item is
``{'im1': [3,h,w] ImageNet-normalised float, 'im1_ori': uint8 HxWx3,
'coord1': SIFT keypoints, 'name1': relative name, 'pad1': (0,0,0,0)}`` with h, w
cropped down to multiples of 16.  The reference ALWAYS runs OpenCV SIFT per
image (only consumed when ``use_sift: True``); OpenCV is not part of this
stack, so ``coord1`` is an empty [0,2] tensor and the Extractor refuses
``use_sift: True`` loudly.  Decoding uses PIL (skimage is absent).
"""
import glob
import os

import numpy as np
import torch
from torch.utils.data import Dataset

MEAN = np.array([0.485, 0.456, 0.406], np.float32)
STD = np.array([0.229, 0.224, 0.225], np.float32)


def to_input(im):
    """uint8 HxWx3 -> (normalised [3,h16,w16] float tensor, cropped uint8 image):
    transforms.ToTensor + Normalize then crop to /16 (hpatches.py:14-17, 35-38)."""
    if im.ndim == 2:
        im = np.stack([im] * 3, -1)
    im = im[..., :3]
    h, w = im.shape[:2]
    im = im[:h - h % 16, :w - w % 16]
    x = (im.astype(np.float32) / np.float32(255.0) - MEAN) / STD
    return torch.from_numpy(np.ascontiguousarray(x.transpose(2, 0, 1))), np.ascontiguousarray(im)


def crop16(im):
    """uint8 HxWx3 -> the cropped (multiples of 16) contiguous uint8 image that
    to_input normalises; the pipelined Extractor uploads this and normalises on
    the device (ops.normalize_rgb8, bit-identical to to_input)."""
    if im.ndim == 2:
        im = np.stack([im] * 3, -1)
    im = im[..., :3]
    h, w = im.shape[:2]
    return np.ascontiguousarray(im[:h - h % 16, :w - w % 16])


def _read(path):
    from PIL import Image
    return np.asarray(Image.open(path).convert("RGB"))


def _ppm_header(f):
    """(width, height, data offset) of a binary RGB PPM (P6, maxval 255) from
    open file ``f``, else None (the caller decodes with PIL)."""
    head = f.read(512)
    if head[:2] != b"P6":
        return None
    vals, i, n = [], 2, len(head)
    while len(vals) < 3:
        while i < n and head[i:i + 1].isspace():
            i += 1
        if i < n and head[i:i + 1] == b"#":   # comment to the end of the line
            while i < n and head[i:i + 1] not in (b"\n", b"\r"):
                i += 1
            continue
        j = i
        while j < n and head[j:j + 1].isdigit():
            j += 1
        if j == i:
            return None
        vals.append(int(head[i:j]))
        i = j
    if i >= n or not head[i:i + 1].isspace() or vals[2] != 255:
        return None
    return vals[0], vals[1], i + 1


class _FileDataset(Dataset):
    """``uint8_only`` (set by the pipelined Extractor): items carry only the
    cropped uint8 image, its name and index -- the float normalisation runs on
    the device, so the loader workers skip it."""

    def __init__(self, configs):
        super().__init__()
        self.configs = configs
        self.imfs = []
        self.uint8_only = False

    def name_of(self, path):
        raise NotImplementedError

    def item_size(self, item):
        """(h, w) of item ``item`` after the crop to multiples of 16, from the
        file header alone (PIL decodes lazily): lets the Extractor size its
        engine workspace and plan its batches before any image is decoded."""
        from PIL import Image
        with Image.open(self.imfs[item]) as im:
            w, h = im.size
        return h - h % 16, w - w % 16

    def item_name(self, item):
        return self.name_of(self.imfs[item])

    def read_into(self, item, out):
        """Decode item ``item`` cropped to multiples of 16 into ``out`` (uint8
        [h16][w16][3], C-contiguous: a slice of the Extractor's pinned staging
        buffer), exactly the bytes crop16(_read(path)) gives.  Binary RGB PPM
        with maxval 255 (HPatches) is raw RGB after its header: the rows are
        read straight into ``out`` (no decode, no intermediate copy when the
        width needs no crop); everything else goes through PIL."""
        path = self.imfs[item]
        h16, w16 = out.shape[0], out.shape[1]
        with open(path, "rb") as f:
            hdr = _ppm_header(f)
            if hdr is not None:
                w, h, off = hdr
                if h - h % 16 == h16 and w - w % 16 == w16:
                    f.seek(off)
                    if w == w16:
                        n = f.readinto(memoryview(out).cast("B"))
                    else:
                        tmp = np.empty((h16, w, 3), np.uint8)
                        n = f.readinto(memoryview(tmp).cast("B"))
                        out[...] = tmp[:, :w16]
                    if n == h16 * w * 3:
                        return
        out[...] = crop16(_read(path))

    def __getitem__(self, item):
        imf = self.imfs[item]
        if self.uint8_only:
            return {"im1_ori": torch.from_numpy(crop16(_read(imf))), "name1": self.name_of(imf),
                    "index": item}
        x, im = to_input(_read(imf))
        return {"im1": x, "im1_ori": im, "coord1": torch.zeros(0, 2), "name1": self.name_of(imf),
                "pad1": (0, 0, 0, 0)}

    def __len__(self):
        return len(self.imfs)


class HPatch_SIFT(_FileDataset):
    """``<data_path>/*/*.ppm``, name = 'seq/idx.ppm' (hpatches.py:19-30)."""

    def __init__(self, configs):
        super().__init__(configs)
        self.imfs = sorted(glob.glob(os.path.join(configs["data_path"], "*", "*.ppm")))

    def name_of(self, p):
        return "/".join(p.split("/")[-2:])


class Aachen_Day_Night(_FileDataset):
    """db/*.jpg, query/*/*/*.jpg, sequences/... (aachen.py:20-47)."""

    def __init__(self, configs):
        super().__init__(configs)
        r = configs["data_path"]
        imfs = glob.glob(os.path.join(r, "db", "*.jpg"))
        imfs += glob.glob(os.path.join(r, "query", "*", "*", "*.jpg"))
        imfs += glob.glob(os.path.join(r, "sequences", "gopro3_undistorted", "*.png"))
        imfs += glob.glob(os.path.join(r, "sequences", "nexus4_sequences", "*", "*.png"))
        self.imfs = sorted(imfs)

    def name_of(self, p):
        s = p.split("/")
        if "db" in s:
            return "/".join(s[-2:])
        if "gopro3_undistorted" in s:
            return "/".join(s[-3:])
        return "/".join(s[-4:])


class ETH_LFB(_FileDataset):
    """<data_path>/<subfolder>/images/* (ETH_local_feature.py:20-31)."""

    def __init__(self, configs):
        super().__init__(configs)
        self.imfs = sorted(glob.glob(os.path.join(configs["data_path"], configs["subfolder"],
                                                  "images", "*")))

    def name_of(self, p):
        return "{}/{}".format(self.configs["subfolder"], os.path.basename(p))


class SyntheticImages(Dataset):
    """Seeded synthetic images for plumbing and benchmarks:
    ``num_images`` uint8 RandomState(1000+i) images of ``height x width``, or
    of ``sizes[i % len(sizes)]`` (a list of [h, w]) for mixed-size streams."""

    def __init__(self, configs):
        super().__init__()
        self.configs = configs
        self.n = int(configs.get("num_images", 8))
        self.h = int(configs.get("height", 480))
        self.w = int(configs.get("width", 640))
        self.sizes = [tuple(int(v) for v in s) for s in configs.get("sizes", None) or []]
        self.uint8_only = False

    def __getitem__(self, item):
        rs = np.random.RandomState(1000 + item)
        h, w = self.sizes[item % len(self.sizes)] if self.sizes else (self.h, self.w)
        raw = rs.randint(0, 256, (h, w, 3)).astype(np.uint8)
        if self.uint8_only:
            return {"im1_ori": torch.from_numpy(crop16(raw)), "name1": "synthetic/%05d.ppm" % item,
                    "index": item}
        x, im = to_input(raw)
        return {"im1": x, "im1_ori": im, "coord1": torch.zeros(0, 2),
                "name1": "synthetic/%05d.ppm" % item, "pad1": (0, 0, 0, 0)}

    def item_size(self, item):
        h, w = self.sizes[item % len(self.sizes)] if self.sizes else (self.h, self.w)
        return h - h % 16, w - w % 16

    def item_name(self, item):
        return "synthetic/%05d.ppm" % item

    def read_into(self, item, out):
        rs = np.random.RandomState(1000 + item)
        h, w = self.sizes[item % len(self.sizes)] if self.sizes else (self.h, self.w)
        out[...] = crop16(rs.randint(0, 256, (h, w, 3)).astype(np.uint8))

    def __len__(self):
        return self.n


class ShardSampler(torch.utils.data.Sampler):
    """Static image sharding for multi-GPU extraction: rank r takes
    {i : i mod world == r} -- no padding, no duplicated images (the
    reference's DistributedSampler pads; extractor.py:95-97)."""

    def __init__(self, n, rank, world):
        self.idx = list(range(rank, n, world))

    def __iter__(self):
        return iter(self.idx)

    def __len__(self):
        return len(self.idx)
