"""CLI drop-in for the reference extract.py (extract.py:1-9):
``python extract.py --config configs/extract_hpatches.yaml [--local_rank r]``.
Multi-GPU: ``torchrun --nproc-per-node N extract.py --config ...`` (one
process per GPU, image-sharded, weights broadcast over RCCL)."""
import argparse

from posfeat_amd.managers.extractor import Extractor

if __name__ == "__main__":
    parser = argparse.ArgumentParser()
    parser.add_argument("--local_rank", type=int, default=-1)
    parser.add_argument("--config", type=str, default="./configs/extract.yaml")
    args = parser.parse_args()
    extractor = Extractor(args)
    extractor.extract()
