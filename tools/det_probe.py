"""Probe: run the config-5 step twice on fresh engines; report grad / forward diffs."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_train_kp import _case
from posfeat_amd.engine import ExtractionEngine
from posfeat_amd.training import KeypointTrainStep
from posfeat_amd.weights import seeded_state_dicts
dev = torch.device("cuda", 0)
d, b, H, W, im1, im2, F1, F2, draws = _case("a")
bb, hd = seeded_state_dicts(0)
res = []
for r in range(2):
    eng = ExtractionEngine(bb, hd, device=dev, train=True)
    st = KeypointTrainStep(eng)
    out, g = st.step(im1.to(dev), im2.to(dev), F1, F2, draws=draws, update=False)
    lp = eng.run(torch.cat([im1, im2]).to(dev), outputs=())["local_point"]
    torch.cuda.synchronize()
    res.append((out.cpu().numpy(), g.cpu().numpy().copy(), lp.cpu().numpy().copy()))
print("autotune", os.environ.get("POSFEAT_AUTOTUNE", "1"),
      "loss diff", np.abs(res[0][0] - res[1][0]).max(),
      "grad diff", np.abs(res[0][1] - res[1][1]).max(), "grad max", np.abs(res[0][1]).max(),
      "lp diff", np.abs(res[0][2] - res[1][2]).max())
