"""The harder-data leg (bench.config_harder: latent 32, M 32, M0 63, efC 512) for each
upper_efc given, at ef 384 / 512 with search_expand 4.
Usage: python tools/harder_probe.py [upper_efc ...]"""
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

for ue in [int(a) for a in sys.argv[1:]] or [0]:
    r = bench.config_harder(torch.device("cuda"), efs=(384, 512), xws=(4,), upper_efc=ue)
    print(json.dumps({"upper_efc": ue, "build_inserts_per_s": r["build_inserts_per_s"],
                      "points": [{k: p[k] for k in ("ef", "recall_at_10", "qps", "roofline_frac")}
                                 for p in r["operating_points"]]}), flush=True)
