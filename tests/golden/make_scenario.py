"""Derive the shipped 3x3 scenario (reference src/sumo_files/scenarios/
grid_3x3.sumocfg -> grid_3x3.net.xml + grid_3x3_p06.rou.xml) into compact data
files with dmdqn_amd.sumo_scenario, so GPU runs (which have no /root/reference)
can use it:
  tests/golden/grid_3x3_p06_scenario.npz   fixture for the loader / parity tests
  config/scenarios/grid_3x3_p06.npz        the same data for train.py --scenario
Run from the repo root: python tests/golden/make_scenario.py"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from dmdqn_amd.sumo_scenario import load_scenario  # noqa: E402

CFG = "/root/reference/src/sumo_files/scenarios/grid_3x3.sumocfg"

if __name__ == "__main__":
    sc = load_scenario(CFG)
    out = os.path.join(ROOT, "tests", "golden", "grid_3x3_p06_scenario.npz")
    sc.save(out)
    dst = os.path.join(ROOT, "config", "scenarios", "grid_3x3_p06.npz")
    shutil.copyfile(out, dst)
    print(f"{sc.rows}x{sc.cols}, {sc.nveh} vehicles, period {sc.period_ms} ms -> {out}, {dst}")
