"""Host-side helpers of bench.py: the sysfs shader-clock reader and the
per-step PMC traffic lookup keyed by the kernel sources."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_clock_sampler_reads_current_level(tmp_path):
    import bench
    f = tmp_path / "pp_dpm_sclk"
    f.write_text("0: 500Mhz\n1: 1600Mhz\n2: 2400Mhz *\n")
    cs = bench.ClockSampler.__new__(bench.ClockSampler)
    cs.path, cs.mhz, cs._stop = str(f), [], None
    assert cs._read() == 2400
    cs.mhz = [2390, 2400, 2380]
    s = cs.summary()
    assert (s["sclk_mhz_min"], s["sclk_mhz_median"], s["sclk_mhz_max"], s["samples"]) == (2380, 2390, 2400, 3)
    cs.mhz = []
    assert cs.summary()["sclk_mhz_median"] is None


def test_traffic_records_match_sources():
    """Every committed per-step traffic record names its profile file, and a
    record is only used while the kernel sources hash the same."""
    import bench
    recs = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic_aux.json")))
    for cfg, r in recs.items():
        assert r["bytes_per_step_scope"] > 0
        assert os.path.exists(os.path.join(ROOT, r["source"].split(" ")[0])), r["source"]
        t, _ = bench.aux_traffic(cfg)
        assert t == (r["bytes_per_step_scope"] if r["source_hash"] == bench.aux_source_hash(cfg) else None)
