"""Where the cond-UNet step's wall time goes, from a rocprofv3 --kernel-trace CSV of the bench (one step between the
last two gradient-norm launches): per stream busy time, the main stream's idle gaps (waits on the weight-gradient
stream or the host), and per-kernel-family time split into "alone on the GPU" vs "overlapped with the other stream".
Usage: python scripts/critical_path.py <run_kernel_trace.csv> [--gaps 25]"""
import argparse
import csv
import re


def family(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    return n[:44]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gaps", type=int, default=25)
    ap.add_argument("--marker", default="norm_finalize_kernel", help="kernel that ends a step (ddpm_prev_kernel: sampling)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    step = rows[marks[-2] + 1: marks[-1] + 1]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = int(step[-1]["End_Timestamp"])
    ks = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, r["Stream_Id"], family(r["Kernel_Name"]),
           (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])) for r in step]
    streams = sorted({k[2] for k in ks}, key=lambda s: -sum(k[1] - k[0] for k in ks if k[2] == s))
    main_s = streams[0]
    print(f"step span {(t1 - t0) / 1e3:.1f} us, {len(ks)} dispatches; main stream {main_s}")
    for s in streams:
        b = sum(k[1] - k[0] for k in ks if k[2] == s)
        print(f"  stream {s}: busy {b / 1e3:.1f} us ({sum(1 for k in ks if k[2] == s)} dispatches)")
    main = [k for k in ks if k[2] == main_s]
    other = [k for k in ks if k[2] != main_s]
    gaps = []
    for p, q in zip(main, main[1:]):
        g = q[0] - p[1]
        if g > 0:
            ov = sum(max(0, min(o[1], q[0]) - max(o[0], p[1])) for o in other)
            gaps.append((g, p[3], q[3], ov, p[1]))
    tot = sum(g[0] for g in gaps)
    print(f"main-stream idle gaps: {tot / 1e3:.1f} us in {len(gaps)} gaps "
          f"(side-stream kernel time inside them {sum(g[3] for g in gaps) / 1e3:.1f} us)")
    for g in sorted(gaps, reverse=True)[:a.gaps]:
        print(f"  {g[0] / 1e3:7.1f} us at {g[4] / 1e3:8.1f}  after {g[1]:<44s} before {g[2]:<44s} side busy {g[3] / 1e3:6.1f}")

    # per family: total, and the part of its time during which the other stream is idle ("alone")
    def overlap(k, ivs):
        return sum(max(0, min(o[1], k[1]) - max(o[0], k[0])) for o in ivs)
    fam = {}
    for k in ks:
        ivs = other if k[2] == main_s else main
        f = fam.setdefault((k[3], k[2] == main_s), [0, 0, 0])
        f[0] += k[1] - k[0]
        f[1] += overlap(k, ivs)
        f[2] += 1
    print("per kernel family (stream M = main, S = side): total, overlapped with the other stream")
    for (n, m), (t, o, c) in sorted(fam.items(), key=lambda kv: -kv[1][0])[:40]:
        print(f"  {'M' if m else 'S'} {t / 1e3:8.1f} us  overlapped {o / 1e3:7.1f}  {c:4d}x  {n}")


if __name__ == "__main__":
    main()
