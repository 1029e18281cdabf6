"""Per-dispatch summary of a rocprofv3 --pmc CSV that holds SQ_WAVES, SQ_INSTS_VALU,
SQ_INSTS_LDS, SQ_WAVE_CYCLES, SQ_WAIT_INST_ANY, SQ_WAIT_ANY, SQ_ACTIVE_INST_VALU,
SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE (tools/gpu_session.sh pmcsq): the clock each
dispatch ran at (GRBM_GUI_ACTIVE / 8 XCDs / duration, MI355X_MICROARCH DVFS note) and
per-wave counts.  Usage: python tools/pmc_clock_summary.py run_counter_collection.csv"""
import csv, sys, collections
for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    d = collections.defaultdict(dict)
    for r in rows:
        key = (r['Dispatch_Id'], r['Kernel_Name'][:28])
        d[key][r['Counter_Name']] = float(r['Counter_Value'])
        d[key]['dur_ns'] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    for (di, k), v in sorted(d.items(), key=lambda x: int(x[0][0])):
        if v['dur_ns'] < 2e6: continue
        ghz = v['GRBM_GUI_ACTIVE'] / 8 / v['dur_ns']
        w = max(1, v['SQ_WAVES'])
        print("%4s %-28s %.3f ms clk %.3f | per wave: VALU %.0f LDS %.0f wave_cyc %.0f wait_inst %.0f wait_any %.0f actVALU %.0f | busy %.3g" % (
            di, k, v['dur_ns']/1e6, ghz, v['SQ_INSTS_VALU']/w, v['SQ_INSTS_LDS']/w, v['SQ_WAVE_CYCLES']/w, v['SQ_WAIT_INST_ANY']/w, v['SQ_WAIT_ANY']/w, v['SQ_ACTIVE_INST_VALU']/w, v['SQ_BUSY_CYCLES']))
