#!/usr/bin/env python3
"""Adds `trace` to tests/golden/notebook_games.json (F1): each rendered game's
DEBUG lines of env.step -- "<name> (player p) plays card c" (env.py:128),
"  ...chooses to replace row r" (env.py:145), "  ...and gains p Hornochsen"
(env.py:165) -- in logged order, parsed from the notebook's stored outputs
(experiments/simple_tournament.ipynb; text only, nothing imported or run).
Run here (where /root/reference exists); the fixture is data."""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NB = "/root/reference/experiments/simple_tournament.ipynb"
FIX = os.path.join(ROOT, "tests", "golden", "notebook_games.json")
KEEP = re.compile(r"\(player \d+\) plays card \d+$|^  \.\.\.chooses to replace row \d+$|^  \.\.\.and gains \d+ Hornochsen$")


def main():
    nb = json.load(open(NB))
    traces = []
    for cell in nb["cells"]:
        if cell.get("cell_type") != "code":
            continue
        text = "".join("".join(o.get("text", "")) for o in cell.get("outputs", []) if o.get("output_type") == "stream")
        if "Dealing cards" not in text:
            continue
        for chunk in text.split("Dealing cards")[1:]:
            lines = []
            for ln in chunk.split("\n"):
                if "The game is over" in ln:
                    break
                ln = ln.rstrip()
                if KEEP.search(ln):
                    lines.append(ln)
            traces.append(lines)
    d = json.load(open(FIX))
    assert len(traces) == len(d["games"]) == 5
    for g, tr in zip(d["games"], traces):
        plays = [ln for ln in tr if "plays card" in ln]
        assert len(plays) == len(g["names"]) * len(g["actions"]), (len(plays), len(g["actions"]))
        g["trace"] = tr
    d["trace_source"] = "DEBUG lines of env.py:128,145,165 in the notebook's rendered games (tools/gen_trace_fixture.py)"
    with open(FIX, "w") as f:
        json.dump(d, f)
    print("traces:", [len(t) for t in traces])


if __name__ == "__main__":
    main()
