import glob, json, sys
for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}/*_n8_*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], "single", d.get("single_gpu_ms"), "slowest", d["slowest_rank_ms"],
          [(v["median_ms"], v["gathers_per_proof"], v["host_gathers_per_proof"]) for v in d["ranks"].values()])
