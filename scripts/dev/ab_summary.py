"""Summarise an A/B log of bench JSON lines: value, operator and precon group rates."""
import json
import sys
from collections import defaultdict

cur, rows = None, defaultdict(list)
for line in open(sys.argv[1]):
    if line.startswith("==="):
        cur = line.split()[1]
    elif line.startswith("{"):
        d = json.loads(line)
        op = d.get("operator_roofline", {}).get("achieved")
        pr = d.get("precon_roofline", {}).get("achieved")
        rows[cur].append((d["value"], op, pr))
for k, v in rows.items():
    print(k, " ".join(f"{a:.1f}" for a, _, _ in v), "| op", " ".join(f"{b:.0f}" for _, b, _ in v if b),
          "| pre", " ".join(f"{c:.0f}" for _, _, c in v if c))
