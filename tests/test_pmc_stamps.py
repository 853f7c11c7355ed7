"""CPU checks of the PMC traffic stamps:

* tools/pmc_traffic.py keeps the kernel clock's instantiations out of a stamp (they
  run only in bench.py's in-step timing graphs; counting them beside the production
  kernels summed two medians per launch -- the tower entries were twice their bytes
  until r06);
* bench.py reports ``traffic`` only for a stamp of its own workload AND library, and
  says why otherwise.
"""
import json
import os
import sys
import types

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)


def test_clocked_instantiations_are_filtered():
    import pmc_traffic as P
    clocked = [
        "void mrec::tower_kernel<8, true, false>(mrec::TowerArgs, mrec::KClock)",
        "void mrec::tower_kernel<8, true, true>(mrec::TowerArgs, mrec::KClock)",
        "void mrec::tower_dw_kernel<4, true, false>(mrec::DwArgs, mrec::KClock)",
        "void mrec::din_att_bwd2_kernel<32, 5, 3, 3, 2, true>(mrec::DinAttArgs, mrec::KClock)",
        "void mrec::din_att_fwd_wave_kernel<32, 5, 3, 3, 2, true>(mrec::DinAttArgs, mrec::KClock)",
        "void mrec::apply_hash_kernel<unsigned short, 4, 2, true>(mrec::BankArgs, long)",
        "void mrec::interact_plan_kernel<unsigned short, 4, true, false, true>(mrec::BankArgs)",
        "void mrec::bucketize_dedup_kernel<true>(mrec::IdsArgs, mrec::RowsArg, long)",
    ]
    production = [
        "void mrec::tower_kernel<8, false, false>(mrec::TowerArgs, mrec::KClock)",
        "void mrec::tower_kernel<8, false, true>(mrec::TowerArgs, mrec::KClock)",
        "void mrec::tower_dw_kernel<4, false, true>(mrec::DwArgs, mrec::KClock)",
        "void mrec::din_att_bwd2_kernel<32, 5, 3, 3, 2, false>(mrec::DinAttArgs, mrec::KClock)",
        "void mrec::apply_hash_kernel<unsigned short, 4, 2, false>(mrec::BankArgs, long)",
        "void mrec::interact_plan_kernel<unsigned short, 4, true, false, false>(mrec::BankArgs)",
        "void mrec::bucketize_dedup_kernel<false>(mrec::IdsArgs, mrec::RowsArg, long)",
        "mrec::bk_apply_kernel<unsigned short, 2>(mrec::BankArgs, mrec::LgWs, mrec::ApplyArgs)",
    ]
    for n in clocked:
        assert P._CLOCKED.search(n), n
    for n in production:
        assert not P._CLOCKED.search(n), n


def test_bench_reports_traffic_only_for_its_workload_and_library(tmp_path, monkeypatch):
    import bench
    args = types.SimpleNamespace(model="deepfm", batch=4096, rows_per_table=38462, zipf=0.0,
                                 shard=False, gpus=1, exchange="auto")
    wl = bench.pmc_workload(args)
    run = {"workload": wl, "lib": "abc", "commit": "c0", "utc": "t",
           "kernels": {"k1": {"hbm_bytes_per_launch": 100}, "k2": {"hbm_bytes_per_launch": 23}}}
    f = tmp_path / "pmc.json"
    f.write_text(json.dumps({"runs": [run]}))
    monkeypatch.setattr(bench, "PMC_FILE", str(f))
    monkeypatch.setattr(bench, "lib_digest", lambda: "abc")
    nbytes, src = bench.pmc_traffic(["k1", "k2"], args)
    assert nbytes == 123 and src["run"]["commit"] == "c0"
    # another library: stale
    monkeypatch.setattr(bench, "lib_digest", lambda: "def")
    nbytes, src = bench.pmc_traffic(["k1"], args)
    assert nbytes is None and src["stale"]["stamped_lib"] == "abc"
    # another workload (Zipf ids): no run for it
    monkeypatch.setattr(bench, "lib_digest", lambda: "abc")
    zargs = types.SimpleNamespace(**dict(vars(args), zipf=1.05))
    nbytes, src = bench.pmc_traffic(["k1"], zargs)
    assert nbytes is None and src["no_run_for"]["zipf"] == 1.05
    # a kernel the stamp does not hold
    nbytes, src = bench.pmc_traffic(["k3"], args)
    assert nbytes is None and src["missing_kernels"] == ["k3"]
