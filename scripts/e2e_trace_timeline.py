"""Timeline of one end-to-end decode phase from a rocprofv3 kernel + memory-copy trace of
netty_amd/e2e_capi (scripts: `rocprofv3 --kernel-trace --memory-copy-trace ... -- netty_amd/e2e_capi
256 256 65535 2 0 256`): per batch stream, the gather, parse, expand, finish kernels and the result
copy, in ms from the phase start, plus the copy engine's busy and idle time.

    python scripts/e2e_trace_timeline.py TRACE_DIR [first_parse_index] [last_parse_index]
"""
import csv
import os
import sys

KEEP = ("k_gather_host", "HOST_TO_DEVICE", "k_parse", "k_expand", "k_decode_fused", "k_dec_finish", "DEVICE_TO_HOST")
DECODE = ("k_parse", "k_decode_fused")


def main():
    d = sys.argv[1]
    a = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    b = int(sys.argv[3]) if len(sys.argv) > 3 else 23
    ev = []
    for k in csv.DictReader(open(os.path.join(d, "tr_kernel_trace.csv"))):
        name = k["Kernel_Name"].split("(")[0].split("::")[-1].replace("void ", "")
        ev.append((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Stream_Id"], name, k["Grid_Size_X"]))
    for m in csv.DictReader(open(os.path.join(d, "tr_memory_copy_trace.csv"))):
        ev.append((int(m["Start_Timestamp"]), int(m["End_Timestamp"]), m["Stream_Id"], m["Direction"].replace("MEMORY_COPY_", ""), ""))
    ev.sort()
    parses = [e for e in ev if e[3] in DECODE and e[4] != "" and int(e[4]) > 64 * 1024] or [e for e in ev if e[3] in DECODE]
    a, b = min(a, len(parses) - 1), min(b, len(parses) - 1)
    t0 = parses[a][0] - 12_000_000
    t1 = parses[b][1] + 30_000_000
    sel = [e for e in ev if t0 <= e[0] <= t1 and e[3] in KEEP]
    base = sel[0][0]
    for e in sel:
        print(f"{(e[0] - base) / 1e6:8.2f} {(e[1] - base) / 1e6:8.2f} {(e[1] - e[0]) / 1e6:6.2f} stream {e[2]} {e[3]} {e[4]}")
    d2h = [e for e in sel if e[3] == "DEVICE_TO_HOST"]
    busy = sum(e[1] - e[0] for e in d2h) / 1e6
    span = (d2h[-1][1] - sel[0][0]) / 1e6
    print(f"result copies: {len(d2h)}, busy {busy:.1f} ms of the phase's {span:.1f} ms")


if __name__ == "__main__":
    main()
