"""Where a live run's time goes (GPU): the default startConsensus of one network,
run to its end, with BENOR_EVENT_STATS set, so the workgroup-batched event
kernel (csrc/benor_event_live.hip) appends its batch counters and the shader
cycles between its control wave's barriers.  One JSON line per (shape, waves):
the kernel's counters, cycles per batch by phase (the phase stamps cost
cycles of their own), and the host's wall time from the start to the final
states, from a run without the counters ("wall_ms") and with them.

    python tools/live_profile.py [--shapes "1024,341;10,5"] [--waves "0,1,3,7,15"] [--forms "default,wave"]
                                 [--k-max 64] [--reps 3] [--vary NAME=v1,v2,...]

waves 0 = the planner's choice (BENOR_LIVE_WAVES unset); forms: BENOR_EVENT_FORM
values, "default" = unset (the register kernel at N <= 16, "wave" the LDS micro-batch one).
--vary: an environment knob set to each value in turn inside every repetition (an
A/B on one box; "-" = unset); the line carries it as "vary".
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ben-or-consensus-algorithm_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="1024,341;1024,512;100,33;10,5;10,4")
    ap.add_argument("--waves", default="0")
    ap.add_argument("--forms", default="default")
    ap.add_argument("--k-max", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--vary", default="")
    a = ap.parse_args()
    fd, path = tempfile.mkstemp(suffix=".jsonl")
    os.close(fd)
    os.environ["BENOR_EVENT_STATS"] = path
    import benor

    vname, vvals = (a.vary.split("=", 1)[0], a.vary.split("=", 1)[1].split(",")) if a.vary else ("", [""])
    for spec in a.shapes.split(";"):
        N, F = (int(x) for x in spec.split(","))
        init = [(i * 7 + 3) % 2 for i in range(N)]
        faulty = [i < F for i in range(N)]
        for form, w in ((f, int(x)) for f in a.forms.split(",") for x in a.waves.split(",")):
            if form == "default":
                os.environ.pop("BENOR_EVENT_FORM", None)
            else:
                os.environ["BENOR_EVENT_FORM"] = form
            if w:
                os.environ["BENOR_LIVE_WAVES"] = str(w)
            else:
                os.environ.pop("BENOR_LIVE_WAVES", None)
            for rep, vv in ((r, v) for r in range(a.reps + 1) for v in vvals):
                if vname and vv == "-":
                    os.environ.pop(vname, None)
                elif vname:
                    os.environ[vname] = vv
                walls = []
                for stats in (False, True):
                    if stats:
                        os.environ["BENOR_EVENT_STATS"] = path
                        open(path, "w").close()
                    else:
                        os.environ.pop("BENOR_EVENT_STATS", None)
                    benor.launchNetwork(N, F, init, faulty)
                    t0 = time.perf_counter()
                    benor.startConsensus(N, seed=rep, k_max=a.k_max)
                    benor.waitConsensus(N)
                    walls.append(time.perf_counter() - t0)
                if rep == 0:
                    continue                            # warm-up (code load, slot allocation)
                lines = [json.loads(x) for x in open(path) if x.strip()]
                s = lines[-1]
                b = max(1, s["batches"])
                out = {"N": N, "F": F, "form": form, "waves": w, **({"vary": f"{vname}={vv}"} if vname else {}), "k_max": a.k_max, "wall_ms": walls[0] * 1e3, "wall_ms_stats": walls[1] * 1e3,
                       "kernel_ms": s["wall_ticks"] / 1e5, "events": s["events"], "batches": s["batches"],
                       "events_per_batch": s["events"] / b, "slots_per_batch": s["batch_slots"] / b,
                       "trigger_batches": s["trigger_batches"], "conflict_cut": s["conflict_cut"],
                       "cross_batches": s["cross_batches"], "cycles_per_batch": s["cycles"] / b,
                       "ns_per_event": s["wall_ticks"] * 10.0 / max(1, s["events"]),
                       "split_cycles_per_batch": {k[4:]: round(s[k] / b, 1) for k in s if k.startswith("cyc_")},
                       "event_wave_per_batch": {k[3:]: round(s.get(k, 0) / b, 1) for k in ("ev_pre", "ev_work", "ev_wait", "ev_drain", "ev_write")}}
                print(json.dumps(out), flush=True)
    os.environ.pop("BENOR_EVENT_STATS", None)
    if vname:
        os.environ.pop(vname, None)
    os.unlink(path)


if __name__ == "__main__":
    main()
