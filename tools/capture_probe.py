"""Probe which multi-stream fork/join patterns survive HIP graph capture (one pattern per process).

Measured on MI355X / ROCm 7 (round 2): patterns whose cross-stream edges all go through the
capturing stream ("hub", "late", "side2side" one way) capture and replay; two side streams that
wait on each other's events ("side2side+bidir", "chain") crash the host in capture_end
(SIGSEGV), and so did a side stream waiting on an event it recorded itself.  The eval
aggregation schedule (aanet_amd/nets/aggregation.py) routes every edge through the capturing
stream for this reason.  Usage: python tools/capture_probe.py [pattern]"""
import subprocess
import sys

import torch


def run(pattern):
    dev = torch.device("cuda")
    main = torch.cuda.current_stream(dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    x = torch.ones(1024, device=dev)

    def body():
        main = torch.cuda.current_stream(dev)
        keep = []
        for st in (s1, s2):
            st.wait_stream(main)
        with torch.cuda.stream(s1):
            a = x * 2
            e1 = torch.cuda.Event()
            e1.record(s1)
        with torch.cuda.stream(s2):
            b = x * 3
            e2 = torch.cuda.Event()
            e2.record(s2)          # never waited on when pattern has "unwaited"
            if "side2side" in pattern:
                s2.wait_event(e1)
                b = b + a
        if "bidir" in pattern:
            e3 = torch.cuda.Event()
            e3.record(s2)
            with torch.cuda.stream(s1):
                s1.wait_event(e3)
                a = a + b
        if "chain" in pattern:  # several rounds of main -> sides -> main
            for _ in range(3):
                eb = torch.cuda.Event()
                eb.record(main)
                with torch.cuda.stream(s1):
                    s1.wait_event(eb)
                    a = a + 1
                    e1 = torch.cuda.Event()
                    e1.record(s1)
                with torch.cuda.stream(s2):
                    s2.wait_event(eb)
                    s2.wait_event(e1)
                    b = b + a
                    e2 = torch.cuda.Event()
                    e2.record(s2)
                with torch.cuda.stream(s1):
                    s1.wait_event(e2)
                    a = a + b
                    e1 = torch.cuda.Event()
                    e1.record(s1)
                main.wait_event(e1)
                main.wait_event(e2)
                keep += [a, b]
        if "hub" in pattern:  # side streams exchange only through the current stream
            for _ in range(3):
                with torch.cuda.stream(s1):
                    a = a + 1
                    e1 = torch.cuda.Event()
                    e1.record(s1)
                with torch.cuda.stream(s2):
                    b = b + 2
                    e2 = torch.cuda.Event()
                    e2.record(s2)
                y0 = x + 5
                main.wait_event(e1)
                main.wait_event(e2)
                ej = torch.cuda.Event()
                ej.record(main)
                y0 = y0 + a + b
                eb = torch.cuda.Event()
                eb.record(main)
                with torch.cuda.stream(s2):
                    s2.wait_event(ej)
                    b = b + a
                    s2.wait_event(eb)
                    b = b + y0
                with torch.cuda.stream(s1):
                    s1.wait_event(eb)
                    a = a + y0 + b
                keep += [a, b, y0]
        keep += [a, b]
        if "unwaited" not in pattern:
            main.wait_event(e2)
        main.wait_event(e1)
        y = x + 1
        if "late" in pattern:  # side work after the main-side join, joined at the end
            eb = torch.cuda.Event()
            eb.record(main)
            with torch.cuda.stream(s1):
                s1.wait_event(eb)
                c = a + y
                keep.append(c)
        for st in (s1, s2):
            main.wait_stream(st)
        return y + a.sum() + b.sum(), keep

    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out, keep = body()
    g.replay()
    torch.cuda.synchronize()
    print(pattern, "ok", out[0].item(), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
    else:
        for p in ("basic", "side2side", "late", "hub", "hub+late"):
            r = subprocess.run([sys.executable, __file__, p], capture_output=True, text=True, timeout=120)
            print(p, "rc", r.returncode, r.stdout.strip()[-200:], r.stderr.strip()[-600:], flush=True)
