"""The harder-data leg (bench.config_harder: latent 32, M 32, M0 63, efC 512) for each
option set given, at ef 384 / 448 / 496 / 512 with search_expand 4.
Usage: python tools/harder_probe.py [name=value:name=value ...]   (e.g. upper_efc=256:batch_ratio_pct=5)"""
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

for spec in sys.argv[1:] or [""]:
    opts = {k: int(v) for k, v in (kv.split("=") for kv in spec.split(":") if kv)}
    r = bench.config_harder(torch.device("cuda"), efs=(384, 512), xws=(4,), fine_efs=(448, 496), opts=opts)
    print(json.dumps({"opts": opts, "build_inserts_per_s": r["build_inserts_per_s"],
                      "points": [{k: p[k] for k in ("ef", "recall_at_10", "qps", "roofline_frac")}
                                 for p in r["operating_points"]]}), flush=True)
