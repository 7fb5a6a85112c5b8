"""Detector configurations the golden fixtures were generated with (shared by
tests/golden/gen_golden.py and the tests; no reference import here)."""

DET_CONFIGS = [
    # name, nms_radius, num_pts, use_nms, thr, thr_mod
    ("hp2048", 1, 2048, True, 0.9, "abs"),      # extract_hpatches.yaml w/ metric num_pts
    ("aachen", 3, 20480, True, 0.5, "abs"),     # extract_aachen.yaml
    ("nothr8192", 1, 8192, True, False, "mean"),
    ("nonms512", 1, 512, False, 0.9, "abs"),
    ("max_r2", 2, 1024, True, 0.5, "max"),
]

CRAFTED_CONFIGS = [("r1", 1, 64, True, False, "mean"),
                   ("r3", 3, 64, True, False, "mean"),
                   ("r2thr", 2, 32, True, 0.5, "abs")]
