"""Memory-subsystem stall counters of one kernel (tools/job.sh step `stall`) folded into
profiles/pmc_cfg<N>.json, beside the traffic counters bench.py's roofline reads.

    python3 tools/pmc_stalls.py gpurun_out/<tag>/stall_cfg<N> <N> [kernel-key]

The summary (tools/pmc_summary.py's summary.json) holds per-launch averages of:
  SQ:   WAVES, WAVE_CYCLES, BUSY_CYCLES, WAIT_ANY, WAIT_INST_ANY, ACTIVE_INST_ANY, INSTS_VALU/SALU/
        VMEM_RD/VMEM_WR/LDS, ACTIVE_INST_VALU/LDS, INST_LEVEL_VMEM
  TA:   BUSY_avr, ADDR_STALLED_BY_TC_CYCLES_sum      TD: TD_BUSY_sum, TC_STALL_sum
  TCP:  PENDING_STALL_CYCLES_sum, TCP_TA_ADDR_STALL_CYCLES_sum, UTCL1_TRANSLATION_MISS_sum,
        UTCL1_STALL_INFLIGHT_MAX_sum                 GRBM: GUI_ACTIVE
Derived (MI355X: 256 CUs, 1,024 SIMDs, 8 XCDs; GRBM_GUI_ACTIVE is summed over the XCDs and the SQ
wave counters count quad-cycles, /opt/skills/guides/MI355X_MICROARCH.md "rocprofv3 PMC slots"):
  cycles            GRBM_GUI_ACTIVE / 8: the kernel's clock cycles
  wait/issue split  WAIT_ANY, WAIT_INST_ANY, ACTIVE_INST_ANY over WAVE_CYCLES (disjoint)
  alu_per_vmem_rd   (VALU + SALU) / VMEM_RD instructions
  valu_issue        VALU instructions per SIMD over its quad-cycles (one wave64 VALU a quad-cycle)
  td_busy, td_tc_stall, tcp_pending_stall, ta_addr_stalled_by_tc: per-CU sums / 256 / cycles
  ta_busy           TA_BUSY_avr / cycles
"""
import json
import os
import sys

CUS, SIMDS, XCDS = 256, 1024, 8


def derive(c):
    g = lambda k: float(c.get(k, 0.0))  # noqa: E731
    cyc = g("GRBM_GUI_ACTIVE") / XCDS
    wc = g("SQ_WAVE_CYCLES")
    out = {
        "cycles": round(cyc),
        "waves": round(g("SQ_WAVES")),
        "wait_any_frac": round(g("SQ_WAIT_ANY") / wc, 4) if wc else None,
        "wait_inst_frac": round(g("SQ_WAIT_INST_ANY") / wc, 4) if wc else None,
        "active_inst_frac": round(g("SQ_ACTIVE_INST_ANY") / wc, 4) if wc else None,
        "insts_valu": round(g("SQ_INSTS_VALU")), "insts_salu": round(g("SQ_INSTS_SALU")),
        "insts_vmem_rd": round(g("SQ_INSTS_VMEM_RD")), "insts_vmem_wr": round(g("SQ_INSTS_VMEM_WR")),
        "insts_lds": round(g("SQ_INSTS_LDS")),
        "alu_per_vmem_rd": round((g("SQ_INSTS_VALU") + g("SQ_INSTS_SALU")) / g("SQ_INSTS_VMEM_RD"), 1)
        if g("SQ_INSTS_VMEM_RD") else None,
        "valu_issue_frac": round(g("SQ_INSTS_VALU") / SIMDS / (cyc / 4), 4) if cyc else None,
        "td_busy_frac": round(g("TD_TD_BUSY_sum") / CUS / cyc, 4) if cyc else None,
        "td_tc_stall_frac": round(g("TD_TC_STALL_sum") / CUS / cyc, 4) if cyc else None,
        "tcp_pending_stall_frac": round(g("TCP_PENDING_STALL_CYCLES_sum") / CUS / cyc, 4) if cyc else None,
        "ta_busy_frac": round(g("TA_BUSY_avr") / cyc, 4) if cyc else None,
        "ta_addr_stalled_by_tc_frac": round(g("TA_ADDR_STALLED_BY_TC_CYCLES_sum") / CUS / cyc, 4)
        if cyc else None,
        "utcl1_translation_misses": round(g("TCP_UTCL1_TRANSLATION_MISS_sum")),
        "utcl1_stall_inflight_max": round(g("TCP_UTCL1_STALL_INFLIGHT_MAX_sum")),
    }
    return out


def main():
    src, cfg = sys.argv[1], int(sys.argv[2])
    want = sys.argv[3] if len(sys.argv) > 3 else None
    summ = json.load(open(os.path.join(src, "summary.json")))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pj = os.path.join(root, "profiles", f"pmc_cfg{cfg}.json")
    d = json.load(open(pj))
    done = []
    for key, ent in d["kernels"].items():
        if want and key != want:
            continue
        name = ent.get("kernel")
        if name not in summ:
            continue
        raw = {k: v for k, v in summ[name].items() if k != "n"}
        ent["stalls"] = dict(derive(raw), raw=raw, source=src)
        done.append((key, name))
    if not done:
        sys.exit(f"no kernel of {pj} in {src}: {sorted(summ)}")
    json.dump(d, open(pj, "w"), indent=1)
    for key, name in done:
        print(key, name, json.dumps({k: v for k, v in d["kernels"][key]["stalls"].items()
                                     if k not in ("raw", "source")}))


if __name__ == "__main__":
    main()
