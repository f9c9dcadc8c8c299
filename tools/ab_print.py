"""One-line summary of a bench JSON line (A/B scripts): label, ms/step, per-class launch ms."""
import json
import sys

d = json.load(open(sys.argv[1]))
r = d["roofline"]
cls = r.get("classes", {r.get("kernel", "main"): r})
print(sys.argv[2], "|", d["ms_per_step"], "ms/step |", d["value"], d["unit"], "|",
      {k: round(v["launch_ms"], 2) for k, v in cls.items()}, flush=True)
