"""Coal-mining disaster dates -> tests/golden/coal_events.json (config C3).

Reads the reference's data file examples/coal/coal.csv (191 numeric lines) the
way examples/coal/coal.jl:383-388 loads it: CSV.read treats line 1 as the
header, so 190 dates remain; they are shifted by their minimum and converted
to days (x 365.25).  T = max (coal.jl:392).  Run once where /root/reference is
mounted; the JSON is the fixture (data only).
"""
import json
import os

SRC = "/root/reference/examples/coal/coal.csv"
HERE = os.path.dirname(os.path.abspath(__file__))

lines = [ln.strip() for ln in open(SRC) if ln.strip()]
dates = [float(x) for x in lines[1:]]  # line 1 is consumed as the CSV header
m = min(dates)
events = [(d - m) * 365.25 for d in dates]
json.dump({"events": events, "T": max(events), "n": len(events),
           "source": "examples/coal/coal.csv via coal.jl:383-392 (header line dropped, (date - min) * 365.25)"},
          open(os.path.join(HERE, "coal_events.json"), "w"), indent=0)
print(len(events), max(events))
