"""Outlier-column counts of every LLM.int8() statistics call (llj_i8_stats, llj_i8_norm_stats) of a
7B llm.int8 decode, per regime of bench.build_model (profiling aid: checks that the C3 regimes of
tools/config_suite.py have the outlier columns they claim).

usage: python tools/i8_outlier_count.py [--outliers random|none|6x20] [--batches 1,8]
"""
import argparse
import collections
import ctypes
import json
import sys
from pathlib import Path

R = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(R))
sys.path.insert(0, str(R / "lit-llama-ja_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from lit_llama import _hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--outliers", default="random")
    ap.add_argument("--batches", default="1,8")
    a = ap.parse_args()
    model = bench.build_model("7B", "llm.int8", outliers=None if a.outliers == "random" else a.outliers)
    orig = _hip.call
    stats = collections.defaultdict(list)
    hip_memcpy = ctypes.CDLL("libamdhip64.so").hipMemcpy

    def count(ws_ptr, M, K):
        torch.cuda.synchronize()
        # i8ws.h: header, the quantized rows, per-(k-block, row) absmax, then the 32 per-block counts
        off_cnt = ((16 + M * K + 15) & ~15) + 4 * 32 * M
        host = (ctypes.c_int * 32)()
        hip_memcpy(host, ctypes.c_void_p(ws_ptr + off_cnt), ctypes.c_size_t(128), 3)
        stats[(M, K)].append(sum(host))

    def call(name, *args):
        r = orig(name, *args)
        if name == "llj_i8_stats":
            count(args[5], args[2], args[3])
        elif name == "llj_i8_norm_stats":
            count(args[7], args[4], args[5])
        return r

    _hip.call = call
    for b in [int(x) for x in a.batches.split(",")]:
        stats.clear()
        bench.time_decode(model, b, 16, 144, 1, 3, 1, use_graph=False)
        print(json.dumps({"regime": a.outliers, "batch": b,
                          **{f"M{k[0]}_K{k[1]}": [min(v), int(sum(v) / len(v)), max(v)] for k, v in stats.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
