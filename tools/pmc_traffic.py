"""Per-launch HBM traffic of one kernel from a prof_summary.py JSON (kernel
trace + FETCH_SIZE + WRITE_SIZE passes of the same bench command), corrected
as MI355X_MICROARCH.md's HBM section prescribes.

usage: python tools/pmc_traffic.py SUMMARY.json KERNEL_PREFIX OUT.json "COMMAND"
"""
import json
import sys


def main():
    src, prefix, out, cmd = sys.argv[1:5]
    d = json.load(open(src))
    stats = {k["name"]: k for x in d for k in x.get("kernel_stats", [])}
    fetch = write = None
    for x in d:
        for k, v in x.get("counters_by_kernel", {}).items():
            if k.startswith(prefix):
                if "FETCH_SIZE" in v:
                    fetch = v["FETCH_SIZE"] / v["dispatches"]
                if "WRITE_SIZE" in v:
                    write = v["WRITE_SIZE"] / v["dispatches"]
    name = [n for n in stats if n.startswith(prefix)][0]
    res = {"kernel": prefix.replace("void ", ""), "command": cmd, "dispatches": stats[name]["calls"],
           "fetch_size_kb_per_launch": round(fetch, 1), "write_size_kb_per_launch": round(write, 1),
           "correction": "FETCH_SIZE is KB (x1024) and on gfx950 reports half the bytes of 16-B/lane reads "
                         "(MI355X_MICROARCH.md HBM section): fetch bytes = 2*1024*FETCH_SIZE; WRITE_SIZE exact: "
                         "1024*WRITE_SIZE",
           "traffic_bytes_per_launch": round(2 * 1024 * fetch + 1024 * write),
           "avg_launch_ns_kernel_trace": stats[name]["avg_ns"]}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
