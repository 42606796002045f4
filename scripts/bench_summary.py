"""One-screen summary of a bench.py JSON line (the last line of the file)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value %.4gG  ms/step %.4f  config %s" % (d["value"] / 1e9, d["ms_per_step"], d["config"].get("workload")))
r = d["roofline"]
print("roofline %s frac %.3f launch %.4f ms  index %s entries, radius %s, build %.0f ms" % (
    r["kernel"], r["frac"], r["launch_ms"], r.get("index_entries"), r.get("index_radius_m"), r.get("index_build_ms", 0)))
print("kernels:", " ".join("%s=%.4f" % (k, v) for k, v in d["kernel_ms"].items()))
h = d.get("host_inclusive")
if h:
    print("host_inclusive %.4gG (%.3f ms, %s B/pt)  soa %.4gG (%.3f ms)" % (
        h["value"] / 1e9, h["ms_per_step"], h.get("input_bytes_per_point"), h["soa"]["value"] / 1e9 if "soa" in h else 0,
        h["soa"]["ms_per_step"] if "soa" in h else 0))
j = d.get("json_report")
if j:
    a = j.get("async") or {}
    print("json_report %.4gM (%.3f ms)  copied %s  async %.4gM best %.4gM  async.copied %s" % (
        j["value"] / 1e6, j["ms_per_call"], "%.4gM" % (j["copied"]["value"] / 1e6) if "copied" in j else "-",
        a.get("value", 0) / 1e6, a.get("best", 0) / 1e6,
        "%.4gM" % (a["copied"]["value"] / 1e6) if "copied" in a else "-"))
c = d.get("cpu_baseline")
if c:
    print("cpu_baseline %.4gM (%s cores)  json_inclusive %s" % (c["value"] / 1e6, c.get("cores"),
          c.get("json_inclusive", {}).get("value") if isinstance(c.get("json_inclusive"), dict) else c.get("json_inclusive")))
ag = d.get("agreement")
if ag:
    v = ag.get("vs_ground_truth", {})
    print("bit_identical %s  seg agreement %.4f interior %.5f outside-outliers %.5f" % (
        ag.get("all_outputs_bit_identical"), v.get("segment_id_agreement", 0), v.get("interior_agreement", 0),
        v.get("interior_agreement_outside_outliers", 0)))
    ds = v.get("datastore_reports")
    if ds:
        print("datastore reports: agreement %.4f interior err %.5f  t0 p50 %.2fs speed p50 %.3f" % (
            ds["report_agreement"], ds["interior_error_rate"], ds["t0_abs_error_s"]["p50"] or 0,
            ds["speed_rel_error"]["p50"] or 0))
