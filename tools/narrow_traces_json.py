"""Per-round phase A / phase B device durations (µs) of default and narrow cfg4 runs from rocprofv3
kernel traces (tools/sessions_scripts/r06_fin3.sh), with medians over the 8-byte rounds (1-14) and
the 4-byte rounds (15 on) of the narrow plan.
usage: python tools/narrow_traces_json.py <session dir> <out.json> <tag>..."""
import csv
import json
import statistics as st
import sys


def phases(path):
    rows = list(csv.DictReader(open(path)))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731
    a = [dur(r) for r in rows if "k_bin_scatter" in r["Kernel_Name"]]
    b = [dur(r) for r in rows if "k_bin_gather" in r["Kernel_Name"]]
    return a, b


def main():
    d, out, tags = sys.argv[1], sys.argv[2], sys.argv[3:]
    res = {"what": "cfg4, tools/bench_configs.py (one warm-up run of 100 FIXED rounds, then the timed run of "
                   "100): per-dispatch durations from rocprofv3 --kernel-trace; rounds of the timed run are "
                   "dispatches 100-199", "runs": {}}
    for t in tags:
        a, b = phases(f"{d}/{t}/run_kernel_trace.csv")
        res["runs"][t] = {
            "phase_a_us": [round(x, 2) for x in a], "phase_b_us": [round(x, 2) for x in b],
            "median_rounds_1_14": {"a": st.median(a[101:115]), "b": st.median(b[101:115])},
            "median_rounds_15_99": {"a": st.median(a[115:200]), "b": st.median(b[115:200])}}
    json.dump(res, open(out, "w"), indent=1)
    for t in tags:
        print(t, res["runs"][t]["median_rounds_1_14"], res["runs"][t]["median_rounds_15_99"])


if __name__ == "__main__":
    main()
