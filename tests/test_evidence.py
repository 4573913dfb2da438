"""The bench line's counter evidence on CPU: profiles/traffic.json entries are
keyed by the measured kernel's code hash, so a kernel that changed after its
PMC run reads null instead of stale bytes, and
scripts/traffic_json.py turns rocprofv3 counter CSVs into HBM bytes and VALU
busy by the formulas DESIGN.md states."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _bench():
    import importlib
    return importlib.import_module("bench")


def test_traffic_lookup_is_keyed_by_code_hash(tmp_path):
    b = _bench()
    from sproxy_amd import md5 as m
    b.m = m                              # bench.py imports the package lazily, in main()
    h = m.kernel_code_hash("md5_fixed_xdma1nt")
    path = tmp_path / "traffic.json"
    ent = {"bytes": 123456, "code_hash": h, "source": "test", "valu_busy": 0.5}
    path.write_text(json.dumps({"entries": {"md5_fixed_xdma1nt@c2@8x16384": ent}}))
    got, note = b.load_traffic(str(path), "md5_fixed_xdma1nt", "c2@8x16384")
    assert got == 123456 and h[:16] in note
    assert b.load_valu_busy(str(path), "md5_fixed_xdma1nt", "c2@8x16384") == 0.5
    # another workload, or the same kernel after a code change: no bytes
    assert b.load_traffic(str(path), "md5_fixed_xdma1nt", "c2@9x16384")[0] is None
    ent["code_hash"] = "0" * 64
    path.write_text(json.dumps({"entries": {"md5_fixed_xdma1nt@c2@8x16384": ent}}))
    got, note = b.load_traffic(str(path), "md5_fixed_xdma1nt", "c2@8x16384")
    assert got is None and note.startswith("stale")
    assert b.load_valu_busy(str(path), "md5_fixed_xdma1nt", "c2@8x16384") is None


def _pmc_csv(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "pmc_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_traffic_json_merges_fetch_write_and_valu_passes(tmp_path):
    k = "md5hip::md5_fixed_xdma1nt(unsigned char const*, unsigned long)"
    fetch, write, valu = (str(tmp_path / x) for x in ("fetch", "write", "valu"))
    # two dispatches, counters summed per dispatch over (here two) XCD rows
    _pmc_csv(fetch, [{"Dispatch_Id": d, "Kernel_Name": k, "Counter_Name": "FETCH_SIZE", "Counter_Value": v}
                     for d, v in ((1, 500.0), (1, 500.0), (2, 600.0), (2, 400.0))])
    _pmc_csv(write, [{"Dispatch_Id": d, "Kernel_Name": k, "Counter_Name": "WRITE_SIZE", "Counter_Value": 16.0}
                     for d in (1, 2)])
    rows = []
    for d in (1, 2):
        rows += [{"Dispatch_Id": d, "Kernel_Name": k, "Counter_Name": "SQ_ACTIVE_INST_VALU",
                  "Counter_Value": 1024 * 1000 / 4 * 0.75},
                 {"Dispatch_Id": d, "Kernel_Name": k, "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": 7.0},
                 {"Dispatch_Id": d, "Kernel_Name": k, "Counter_Name": "GRBM_GUI_ACTIVE", "Counter_Value": 8000.0}]
    _pmc_csv(valu, rows)
    out = tmp_path / "traffic.json"
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "traffic_json.py"), fetch, write,
                        "c2@8x16384", "--valu", valu, "--out", str(out), "--source", "test"],
                       capture_output=True, text=True, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    e = json.loads(out.read_text())["entries"]["md5_fixed_xdma1nt@c2@8x16384"]
    assert e["read_bytes"] == 2 * 1024 * 1000 and e["write_bytes"] == 1024 * 16
    assert e["bytes"] == e["read_bytes"] + e["write_bytes"] and e["dispatches"] == 2
    assert abs(e["valu_busy"] - 0.75) < 1e-9 and e["gpu_cycles"] == 1000
    from sproxy_amd import md5 as m
    assert e["code_hash"] == m.kernel_code_hash("md5_fixed_xdma1nt")


def test_cited_evidence_exists():
    """Every `profiles/...` file the docs cite is in the tree, and every
    `scripts/...` path they cite is either in the tree or in
    scripts/README.md's table of deleted scripts (recoverable from git)."""
    import glob
    import re
    deleted = open(os.path.join(REPO, "scripts", "README.md")).read()
    missing = []
    for doc in ("DESIGN.md", "INTEGRATION.md", "README.md", "DESIGN_HISTORY.md",
                os.path.join("profiles", "README.md")):
        text = open(os.path.join(REPO, doc)).read()
        for ref in set(re.findall(r"`((?:profiles|scripts)/[^`\s]+)`", text)):
            p = ref.split("::")[0].rstrip(".,;:")
            if "{" in p or "<" in p or ".." in p or (p.startswith("scripts/") and "*" in p):
                continue                                  # a family of files, not one path
            if glob.glob(os.path.join(REPO, p)):
                continue
            base = os.path.basename(p.rstrip("/"))
            listed = f"`{os.path.splitext(base)[0]}`" in deleted or base in deleted
            if p.startswith("scripts/") and listed:
                continue                                  # deleted; recoverable from git
            missing.append((doc, p))
    assert not missing, missing
