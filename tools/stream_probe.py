"""Diagnostic: bench.py's HBM streaming probe alone (bench.stream_probe) on
the current device, printed as one JSON line.  usage: python tools/stream_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

s = torch.cuda.Stream()
print(json.dumps(bench.stream_probe(s)))
