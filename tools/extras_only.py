#!/usr/bin/env python3
"""Run only bench.py's config-3 (MCS) and config-4 (PUCT) legs -- the target
of the SQ / kernel-trace passes in tools/sq_extras.sh.
Usage: python tools/extras_only.py [mcs|puct|both]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "both"
    import torch

    torch.cuda.set_device(0)
    out = {}
    if which in ("mcs", "both"):
        out["mcs"] = bench.bench_mcs(8192, 256)
    if which in ("puct", "both"):
        out["puct"] = bench.bench_puct(8192)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
