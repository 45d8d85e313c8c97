"""One summary line of a bench.py JSON output (A/B scripts under tools/)."""
import json
import sys


def last_json(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


def main():
    kind, path, tags = sys.argv[1], sys.argv[2], " ".join(sys.argv[3:])
    r = last_json(path)
    if kind == "head":
        roof = r["roofline"]
        conc = roof["concurrent"] or {}
        print(tags, round(r["value"] / 1e9, 3), "G ms", round(r["ms_per_step"], 4), "k_play",
              round(roof["kernel_ms"] * 1e3, 1), "ahead", round((conc.get("kernel_ms") or 0) * 1e3, 1),
              "decode", round((conc.get("decode_kernel_ms") or 0) * 1e3, 1))
    elif kind == "puct":
        x = r["extra_config4_puct"]
        print(tags, round(x["value"] / 1e6, 1), "M playout env-steps/s wall", round(x["wall_s"], 3), x["mlp"])
    elif kind == "mixed":
        x = r["extra_config5_run_py_league"]
        print("run.py league s/round", round(x["s_per_round"], 3))
        print(json.dumps(x.get("phases")))
    else:
        raise SystemExit(f"unknown kind {kind}")


if __name__ == "__main__":
    main()
