cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/wkt
SDZ_WDEC=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/wkt -o run --output-format csv -- python3 tools/run_c2.py --mode inflate --steps 1 > gpurun_out/wkt/log 2>&1 || exit 1
f=$(find gpurun_out/wkt -name "run_kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n=r["Kernel_Name"].split("(")[0]
    if "inflate" in n or "resolve" in n:
        print(n, (int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e6, "ms", r.get("Workgroup_Size_X",""), r.get("Grid_Size_X",""))
PY
