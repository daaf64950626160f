"""List the dispatches of a rocprofv3 kernel_trace.csv in order: kernel (short name), grid x, workgroup
x, LDS bytes, duration ms, start offset ms.  Optional substrings filter the kernels.
Usage: python scripts/trace_list.py <kernel_trace.csv> [substring ...]"""
import csv
import sys


def main():
    path, keys = sys.argv[1], sys.argv[2:]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t0 = int(rows[0]["Start_Timestamp"]) if rows else 0
    for r in rows:
        name = r["Kernel_Name"]
        if keys and not any(k in name for k in keys):
            continue
        short = name.split("(")[0][-60:]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{short:60s} grid {r.get('Grid_Size_X', r.get('Grid_Size', '?')):>9s} wg {r.get('Workgroup_Size_X', '?'):>4s} "
              f"lds {r.get('Group_Segment_Size', r.get('LDS_Block_Size', '?')):>6s} {(e - s) / 1e6:9.3f} ms  @ {(s - t0) / 1e6:10.3f}")


if __name__ == "__main__":
    main()
