"""Run bench.config_legs alone (profiling helper)."""
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402
print(json.dumps(bench.config_legs(torch.device("cuda", 0))))
