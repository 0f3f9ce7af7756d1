"""BASELINE configs[2] alone (1M x 768 Euclidean batched insert at efConstruction 64,
bench.config2): the build a rocprofv3 --pmc pass of tools/profile_round.sh measures
for configs[2]'s roofline.traffic.  Usage: python tools/config2_probe.py [build_expand]"""
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

xw = int(sys.argv[1]) if len(sys.argv) > 1 else 4
print(json.dumps(bench.config2(torch.device("cuda"), xw, pmc_json="")), flush=True)
