#!/usr/bin/env python3
"""Per-block timeline of one traced forward (rocprofv3 --kernel-trace CSV): for each DiT block,
the image-stream (main) and text-stream (side) kernels with start offsets and durations, and the
gap before each attention launch (time the main stream waited on the side stream's text QKV).
    python tools/timeline.py gpurun_out/<tag>/trace/run_kernel_trace.csv [forward_index]"""
import csv
import sys


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:34]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    fi = int(sys.argv[2]) if len(sys.argv) > 2 else -2
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    att = [i for i, r in enumerate(rows) if "attn_pp_kernel" in r["Kernel_Name"]]
    nfwd = len(att) // 60
    blocks = att[(nfwd + fi) * 60 if fi < 0 else fi * 60:][:60]
    gaps = []
    for bi in range(1, 60):
        a0, a1 = blocks[bi - 1], blocks[bi]
        seg = rows[a0 + 1:a1]
        main_end = max((int(r["End_Timestamp"]) for r in seg if int(r["Queue_Id"]) == int(rows[a1]["Queue_Id"])),
                       default=int(rows[a0]["End_Timestamp"]))
        gaps.append((int(rows[a1]["Start_Timestamp"]) - main_end) / 1e3)
        if bi in (1, 30):
            t0 = int(rows[a0]["Start_Timestamp"])
            print(f"--- block {bi}: kernels between attention {bi - 1} and {bi} (us from attention start)")
            for r in [rows[a0]] + seg + [rows[a1]]:
                s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
                print(f"  q{r['Queue_Id']:>2} {short(r['Kernel_Name']):34s} {s / 1e3:9.1f} .. {e / 1e3:9.1f}  ({(e - s) / 1e3:7.1f})")
    per = (int(rows[blocks[-1]]["Start_Timestamp"]) - int(rows[blocks[0]]["Start_Timestamp"])) / 59 / 1e3
    print(f"block period {per:.1f} us; attention start waited on a non-main kernel: mean {sum(gaps) / len(gaps):.1f} us, "
          f"max {max(gaps):.1f} us")


if __name__ == "__main__":
    main()
