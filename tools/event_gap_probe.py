"""Cost of a torch.cuda.Event record between two dependent kernels on one stream (the ~6 us gaps the
C2 step timelines show after cf_begin and bits_list, both followed by an event record).

Times N tiny kernels back to back, then the same with an event recorded after each, and with a
record every other kernel; prints us per kernel for each form.  Measured (r06, profiles/r06_event_gap.json):
1.7 us per kernel plain, 6.7 with a record after each -- the same with a device-scope-release event
(hipEventReleaseToDevice): the cost is the marker packet, not the fence.   python3 tools/event_gap_probe.py"""
import json
import sys

import torch


def run(n: int, form: str) -> float:
    x = torch.zeros(1, device="cuda")
    ev = torch.cuda.Event()
    tev = torch.cuda.Event(enable_timing=True)
    # host far ahead: queue everything behind a long kernel so launch cost never shows
    big = torch.empty(1 << 28, device="cuda")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(12):
        big.fill_(1.0)
    e0.record()
    for i in range(n):
        x.add_(1.0)
        if form == "event":
            ev.record()
        elif form == "timing_event":
            tev.record()
        elif form == "event_half" and i % 2 == 0:
            ev.record()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / n


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    out = {}
    for rep in range(3):
        for form in ("plain", "event", "event_half", "timing_event"):
            out.setdefault(form, []).append(round(run(n, form), 2))
    print(json.dumps({"us_per_kernel": out, "n": n}))


if __name__ == "__main__":
    main()
