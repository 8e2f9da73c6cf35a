"""Print the headline, secondaries and host split of bench JSON lines (round-6 sessions)."""
import json
import sys

for path in sys.argv[1:]:
    lines = [x for x in open(path) if x.startswith("{")]
    if not lines:
        print(path, "no JSON line")
        continue
    d = json.loads(lines[-1])
    c = d.get("config", {})
    print(path, "value %.2f G" % (d["value"] / 1e9), "ms %.4f" % d["ms_per_step"], "p50", d.get("p50_rtt_us"),
          "host_split", c.get("host_split"), "host_us", c.get("host_us_per_step"))
    for k, v in d.get("secondaries", {}).items():
        if isinstance(v, dict) and "value" in v:
            print("  %-20s %8.2f G  %.4f ms" % (k, v["value"] / 1e9, v.get("ms_per_step", 0)))
        elif isinstance(v, dict):
            print("  %-20s %s" % (k, str(v)[:200]))
