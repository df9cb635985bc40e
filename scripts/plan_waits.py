"""Every cross-stream wait the recorded cond-UNet (or DiT) step puts on its MAIN stream, in issue order: the main-stream
kernel before and after the wait, and the stream and last kernel the awaited event follows. Read beside
scripts/critical_path.py's main-stream idle gaps ("after X before Y"): a gap behind a wait whose producer finished long
before is the wait's own cost, a gap with side-stream work inside it is a real dependency.
Usage: python scripts/plan_waits.py [--workload cond-unet|dit|uncond-unet]"""
import argparse
import collections
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "stablediffusion-pytorch_amd"), REPO]
import torch  # noqa: E402

from scripts.device_step import make  # noqa: E402


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:58]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cond-unet")
    a = ap.parse_args()
    from sdmi import _lib, plan as P, streams
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    streams.reserve(dev, n=streams.workload_streams(a.workload))
    log = []  # (kind, stream, event) of every event record / wait, in plan order
    rec, wait = P.record_event, P.wait_event

    def rec_hook(ev, stream):
        r = rec(ev, stream)  # (a torch event gets its HIP handle at its first record)
        if P.RECORDING is not None:
            log.append(("rec", stream.cuda_stream, ev.cuda_event))
        return r

    def wait_hook(stream, ev):
        if P.RECORDING is not None:
            log.append(("wait", stream.cuda_stream, ev.cuda_event))
        return wait(stream, ev)

    P.record_event, P.wait_event = rec_hook, wait_hook
    cap = make(a.workload, dev)  # records the plan (the hooks see the recording's edges)
    P.record_event, P.wait_event = rec, wait
    plan = cap.plan
    L = _lib.lib()
    n = plan.info()[0]
    kind, name, st = ctypes.c_int(), ctypes.c_char_p(), ctypes.c_void_p()
    ops = []
    for i in range(n):
        _lib.check(L.sdmi_plan_op_info(plan.handle, i, ctypes.byref(kind), ctypes.byref(name), None, None, None), "info")
        _lib.check(L.sdmi_plan_op_stream(plan.handle, i, ctypes.byref(st)), "stream")
        ops.append((kind.value, st.value or 0, name.value.decode(errors="replace") if name.value else ""))
    names = subprocess.run(["c++filt"], input="\n".join(o[2] or "-" for o in ops), capture_output=True,
                           text=True).stdout.splitlines()
    ops = [(k, s, short(nm) if k == 0 else "") for (k, s, _), nm in zip(ops, names)]
    # the recording's own log is in step with the plan's event / wait ops (the first steps' log entries precede it)
    edges = [o for o in ops if o[0] in (1, 2)]
    log = log[len(log) - len(edges):]
    streams_seen = collections.Counter(s for k, s, _ in ops if k == 0)
    main = streams_seen.most_common(1)[0][0]
    sid = {s: i for i, (s, _) in enumerate(streams_seen.most_common())}
    last_kernel = {}
    event_src = {}  # event -> (stream, last kernel on it when recorded)
    # events recorded LATER in the plan than a wait on them: the previous replay's record (the optimizer chunks of step
    # N - 1 that step N's forward waits for); their producers, from a first pass over the plan
    later_src, lk, lj = {}, {}, 0
    for k, s, nm in ops:
        if k == 0:
            lk[s] = nm
        elif k in (1, 2):
            _, _, ev = log[lj]
            lj += 1
            if k == 1:
                later_src[ev] = (sid.get(s, -1), "previous step: " + lk.get(s, "(none)"))
    li = 0
    prev_main = "-"
    pending = []
    print(f"{n} ops; streams by launches: " + ", ".join(f"s{sid[s]}={c}" for s, c in streams_seen.most_common()))
    print("main-stream waits: <main kernel before> | waits on s<k> after <producer kernel> | <main kernel after>")
    count = collections.Counter()
    for k, s, nm in ops:
        if k == 0:
            last_kernel[s] = nm
            if s == main:
                for w in pending:
                    print(f"  {prev_main:58s} | s{w[0]} after {w[1]:50s} | {nm}")
                    count[(w[0], w[1][:30])] += 1
                pending = []
                prev_main = nm
            continue
        if k not in (1, 2):
            continue
        kind_s, stream_s, ev = log[li]
        li += 1
        if k == 1:
            event_src[ev] = (sid.get(s, -1), last_kernel.get(s, "(none)"))
        elif s == main:
            src = event_src.get(ev) or later_src.get(ev, (-1, "(recorded before the plan)"))
            if src[0] != sid[main]:
                pending.append(src)
    print(f"{sum(count.values())} cross-stream waits on the main stream")


if __name__ == "__main__":
    main()
