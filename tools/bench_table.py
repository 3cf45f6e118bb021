"""DESIGN.md §7's per-configuration table from a directory of bench.py lines.
usage: python tools/bench_table.py profiles/r05/final/bench"""
import json
import sys

B = sys.argv[1].rstrip("/") + "/"
ROWS = [("rmsc03 (headline, configs[1])", "rmsc03"), ("rmsc03_rl (GymKernel + DummyRL, configs[3] shape)", "rmsc03_rl"),
        ("rmsc03_ddqn (+ PyTorch DDQN learner, configs[3])", "rmsc03_ddqn"),
        ("rmsc03_sweep (scripts/rmsc03.sh options, §1k)", "rmsc03_sweep"), ("rmsc01 (§1b)", "rmsc01"),
        ("rmsc02 (§1c)", "rmsc02"), ("obi_rmsc02 (§1c)", "obi_rmsc02"), ("random_fund_value (§1e)", "random_fund_value"),
        ("random_fund_diverse (§1e)", "random_fund_diverse"), ("hist_fund_value (§1f)", "hist_fund_value"),
        ("hist_fund_diverse (§1f)", "hist_fund_diverse"), ("marketreplay IBM 2003-01-14 (configs[4] shape)", "marketreplay"),
        ("marketreplay GOOG 2012-06-21", "marketreplay_GOOG_2012-06-21"), ("sparse_zi_1000 (configs[2])", "sparse_zi_1000"),
        ("sparse_zi_100", "sparse_zi_100"), ("value_noise", "value_noise"), ("rmsc03_sbmm (§1j, subscribe)", "rmsc03_sbmm"),
        ("rmsc03_sbmm_poll (§1j)", "rmsc03_sbmm_poll")]


def line(c):
    f = B + ("bench_%s.json" % c if c.startswith("marketreplay_") else "bench_%s_default.json" % c)
    return json.loads(open(f).read().strip().splitlines()[-1])


def rate(v):
    return "%.2f G" % (v / 1e9) if v >= 1e9 else "%.0f M" % (v / 1e6)


for name, c in ROWS:
    d = line(c)
    r, cb = d["roofline"], d["cpu_baseline"]
    kern = r["kernel"].split("<")[0].replace("mxa_", "").replace("_kernel", "")
    ms = r["avg_launch_ms"]
    kms = "%s %s ms" % (kern, ("%.3g" % ms) if ms < 100 else "%.0f" % ms)
    if kern == "step":
        kms += " × %d" % (r["launches"] // d["steps"])
    pmc = r.get("traffic_per_event")
    match = r.get("traffic_record", {}).get("match")
    lb = r.get("latency_bound", {}).get("frac")
    print("| %s | %d | **%s** | %.1f | %s | %.0f, %.4f (%.4f) | %s | %s | %.0f M / %.0f M |" % (
        name, d["config"]["envs_per_gpu"], rate(d["value"]), d["ms_per_step"], kms, r["algo_bytes_per_event"], r["frac"],
        r.get("strict", {}).get("frac", r["frac"]), ("%.0f" % pmc if pmc else "—") + ("" if match else " (no record)"),
        "%.2f" % lb if lb else "—", cb["value"] / 1e6, cb["single_thread"]["value"] / 1e6))
print()
print("`step`/s: " + ", ".join("%s %.2f M" % (c, line(c)["config"]["gym_steps_per_s"] / 1e6)
                              for c in ("rmsc03_rl", "rmsc03_ddqn", "marketreplay", "marketreplay_GOOG_2012-06-21")) + ".")
