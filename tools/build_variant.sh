#!/bin/bash
# Build a measurement variant of libwcg.so: tools/build_variant.sh NAME [SRC_ROOT] -- [-DFLAG=V ...]
# Output build/var/libwcg_NAME.so; refuses (deletes) a library whose k_map breaks the in-flight
# register discipline (tools/check_inflight.py) - such a build reads stale prefetch registers.
set -e
NAME=$1; shift
SRC=/root/repo
if [ "$1" != "--" ] && [ -n "$1" ]; then SRC=$1; shift; fi
[ "$1" == "--" ] && shift
OUT=/root/repo/build/var/libwcg_$NAME.so
mkdir -p /root/repo/build/var
cd /tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -fvisibility=hidden -pthread "$@" \
  -o $OUT $SRC/mit-6.824-2015_amd/csrc/wcg_api.hip -L/opt/rocm/lib -lrccl 2>&1 | grep -v hip-link || true
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S "$@" -o /tmp/var_$NAME.s \
  $SRC/mit-6.824-2015_amd/csrc/wcg_api.hip 2>/dev/null
python3 - "$NAME" <<'PY'
import sys, os
sys.path.insert(0, "/root/repo/tools")
import check_inflight
name = sys.argv[1]
text = open(f"/tmp/var_{name}.s").read()
e = []
for sym in ("_ZN3wcg5k_mapILi0ELb1EEEvNS_7MapArgsE", "_ZN3wcg5k_mapILi0ELb0EEEvNS_7MapArgsE", "_ZN3wcg5k_aggILi0EEEvNS_7AggArgsENS_7MapArgsE", "_ZN3wcg5k_aggILi1EEEvNS_7AggArgsENS_7MapArgsE"):
    e += check_inflight.check(text, sym)[0]
if e:
    os.remove(f"/root/repo/build/var/libwcg_{name}.so")
    print(f"variant {name}: REFUSED (in-flight discipline):", *e[:3], sep="\n  ")
    sys.exit(1)
print(f"variant {name}: ok")
PY
