"""Pair a configs.jsonl (tools/configs.sh) with counter stamps taken afterwards on the same library.

tools/gpu_round.sh runs the PMC passes and the config lines in one GPU call, so the lines print
before profiles/pmc_traffic.json, pmc_valu.json and isa_mix.json hold this library's entries,
and their `roofline.traffic` / `roofline.secondary` counters read null.  This fills them in
with bench.py's own code (load_traffic / load_valu / load_isa_mix, secondary_block), from each
line's own launch time (`roofline.kernel_avg_ms`), only when every stamp names the library the
line ran on (the sha written by that run, <run dir>/lib_sha16.txt), and marks the line
`"restamped": true`.  Nothing else in a line changes.

    python tools/restamp_configs.py <configs.jsonl> <lib_sha16.txt> <out.jsonl>
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

CODES_S = {7: 6, 9: 8}


def main():
    src, sha_file, out = sys.argv[1:4]
    sha = open(sha_file).read().split()[-1].strip()
    if bench.lib_sha16() != sha:
        raise SystemExit(f"the library here ({bench.lib_sha16()}) is not the one the lines ran on ({sha})")
    lines = []
    for raw in open(src):
        d = json.loads(raw)
        cfg, rf = d["config"], d["roofline"]
        K = 9 if "K=9" in cfg["workload"] else 7
        soft = "soft" in cfg["workload"]
        F, L = cfg["frames_per_gpu"], cfg["frame_bits"]
        key = f"K{K}_{'soft' if soft else 'hard'}_F{F}_L{L}"
        kernel = rf["secondary"]["kernel"]
        avg_ms = rf["kernel_avg_ms"]
        state_steps = F * (1 << CODES_S[K]) * (L + CODES_S[K])
        traffic = bench.load_traffic(key)
        rf["traffic"] = traffic
        rf["secondary"] = bench.secondary_block(avg_ms, state_steps, kernel, bench.load_valu(key),
                                                bench.load_isa_mix(kernel, soft))
        d["restamped"] = True
        lines.append(d)
        print(cfg.get("baseline_config"), key, kernel, "traffic", traffic, "valu frac",
              rf["secondary"].get("frac"), "issue_priced frac", rf["secondary"].get("issue_priced", {}).get("frac"))
    with open(out, "w") as fh:
        for d in lines:
            fh.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
