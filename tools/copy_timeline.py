#!/usr/bin/env python3
"""Host-to-device copy timeline of a rocprofv3 --memory-copy-trace run.

    python tools/copy_timeline.py <run_memory_copy_trace.csv> <run_kernel_trace.csv> [gap_us]

Splits the trace into calls (H2D copies separated by more than gap_us, default
500 us, of idle link), then for each call prints its span, the time at least
one copy of more than 100 us was moving, the time two or more such copies
overlapped, the longest idle gap between them, and the copies themselves
(start, duration, stream) for the last call.
"""
import csv
import sys


def main():
    copies = [r for r in csv.DictReader(open(sys.argv[1])) if "HOST_TO_DEVICE" in r["Direction"]]
    gap = float(sys.argv[3]) if len(sys.argv) > 3 else 500.0
    szk = next((k for k in (copies[0].keys() if copies else []) if "size" in k.lower() or "bytes" in k.lower()), None)
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r.get("Stream_Id", "") + (f" {int(r[szk]) / 1e6:8.1f} MB {int(r[szk]) / max(1, int(r['End_Timestamp']) - int(r['Start_Timestamp'])):6.1f} GB/s" if szk else ""))
                for r in copies)
    calls, cur, end = [], [], None
    for s, e, st in ev:
        if cur and (s - end) / 1e3 > gap:
            calls.append(cur)
            cur = []
        cur.append((s, e, st))
        end = e if end is None else max(end, e)
    if cur:
        calls.append(cur)
    for ci, c in enumerate(calls):
        big = [(s, e) for s, e, _ in c if (e - s) / 1e3 > 100]
        t0, t1 = c[0][0], max(e for _, e, _ in c)
        pts = sorted([(s, 1) for s, _ in big] + [(e, -1) for _, e in big])
        busy = over = 0.0
        depth, last = 0, None
        for t, d in pts:
            if last is not None:
                if depth >= 1:
                    busy += t - last
                if depth >= 2:
                    over += t - last
            depth += d
            last = t
        idle = [(b[0] - a[1]) / 1e3 for a, b in zip(sorted(big), sorted(big)[1:]) if b[0] > a[1]]
        print(f"call {ci}: span {(t1 - t0) / 1e3:8.1f} us, copies {len(c)}, big {len(big)}, "
              f"link busy {busy / 1e3:8.1f} us, >=2 big copies at once {over / 1e3:8.1f} us, "
              f"largest idle gap {max(idle) if idle else 0:6.1f} us")
    last = calls[-1]
    t0 = last[0][0]
    print("last call's copies: start_us dur_us stream [MB GB/s]")
    for s, e, st in last:
        print(f"  {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {st}")


if __name__ == "__main__":
    main()
