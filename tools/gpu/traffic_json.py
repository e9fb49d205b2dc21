"""HBM bytes per launch of the bench's isolated roofline call (64,512 sets) from the PMC passes
of tools/gpu/pmc.sh (its summary.json): (FETCH_SIZE x 2 + WRITE_SIZE) x 1024 per dispatch
(rocprofv3 reports KB; on gfx950 FETCH_SIZE counts half the bytes of wide reads,
MI355X_MICROARCH.md "HBM"), with the kernel metadata beside it.  bench.py reads the output
(TRAFFIC_FILE).

    python tools/gpu/traffic_json.py gpurun_out/<tag>/pmc/summary.json profiles/<round>/traffic.json
"""
import json
import sys

SETS = 64512


def per(d, k):
    c = d.get(k) or {}
    if not c:
        return None
    w = c.get("SQ_WAVES") or 1
    cyc = c.get("SQ_WAVE_CYCLES") or 1
    return {"bytes_per_launch": (c.get("FETCH_SIZE", 0) * 2 + c.get("WRITE_SIZE", 0)) * 1024,
            "valu_insts_per_wave": c.get("SQ_INSTS_VALU", 0) / w,
            "wait_any_per_wave_cycle": c.get("SQ_WAIT_ANY", 0) / cyc,
            "valu_active_per_wave_cycle": c.get("SQ_ACTIVE_INST_VALU", 0) / cyc}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    s = json.load(open(src))
    d, meta = s["per_dispatch"], s.get("kernel_meta", {})
    out = {"note": "HBM bytes per launch of the bench's isolated roofline call (%d sets): (FETCH_SIZE x 2 + "
                   "WRITE_SIZE) x 1024 from the PMC passes of tools/gpu/pmc.sh over tools/gpu/roof_call.py "
                   "(source: %s); k_miller = the Miller stage's k_lines + k_facc" % (SETS, src),
           "source": src}
    kp = per(d, "k_prep")
    if kp:
        kp["sets"] = SETS
        kp["scratch_bytes_per_lane"] = int((meta.get("k_prep") or {}).get("scratch") or 0)
        out["k_prep"] = kp
    kl, kf = per(d, "k_lines"), per(d, "k_facc")
    if kl and kf:
        out["k_miller"] = {"sets": SETS, "bytes_per_launch": kl["bytes_per_launch"] + kf["bytes_per_launch"],
                           "kernels": {"k_lines": dict(kl, scratch_bytes_per_lane=int((meta.get("k_lines") or {}).get("scratch") or 0)),
                                       "k_facc": dict(kf, scratch_bytes_per_lane=int((meta.get("k_facc") or {}).get("scratch") or 0))}}
    fin = per(d, "k_final12")
    if fin:
        fin["sets"] = SETS
        out["k_final"] = fin
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: round(v["bytes_per_launch"] / 1e9, 3) for k, v in out.items() if isinstance(v, dict)}))


if __name__ == "__main__":
    main()
