#!/usr/bin/env bash
# The node-agent image's ROCm runtime: copy the libraries the agent loads (libamd_smi,
# dlopen'd; the diagnostics library, which links the HIP runtime) and, to a fixpoint,
# every library they need from /opt/rocm, into OUT.  Used by the Dockerfile's node-agent
# stage and by tests/gpu/test_node_image_closure.py, which runs the agent's diagnostics
# with only OUT on the library path and checks that nothing else came from /opt/rocm.
#
#   tools/node_image_closure.sh OUT DIAG_LIB [ROCM=/opt/rocm]
#
# Non-ROCm dependencies (libdrm, libdrm_amdgpu, libnuma, libelf, libssl) come from the
# image's base packages (Dockerfile: libdrm2 libdrm-amdgpu1 libnuma1 libelf1 libssl3).
set -euo pipefail
out=${1:?out dir}; diag=${2:?diagnostics library}; rocm=${3:-/opt/rocm}
mkdir -p "$out"
cp -L "$rocm/lib/libamd_smi.so" "$diag" "$out/"
# Libraries loaded with dlopen, by their sonames, so ldd does not list them (found by
# the loader trace in tests/gpu/test_node_image_closure.py):
#   libamd_comgr.so.N              the HIP runtime's code-object manager (~160 MB: one copy)
#   libhsa-amd-aqlprofile64.so     the HSA runtime's profiling extension (opened by its
#                                  unversioned name)
#   librocprofiler-sdk-roctx.so.1  the agent's own roctx ranges (native/core/roctx.cc)
for f in "$rocm"/lib/libamd_comgr.so.[0-9] "$rocm"/lib/libhsa-amd-aqlprofile64.so \
         "$rocm"/lib/librocprofiler-sdk-roctx.so.[0-9]; do
  [ -e "$f" ] && cp -L "$f" "$out/"
done
while :; do
  added=0
  for f in "$out"/*.so*; do
    while read -r dep; do
      base=$(basename "$dep")
      if [ ! -e "$out/$base" ]; then
        cp -L "$dep" "$out/$base"
        added=1
      fi
    done < <(ldd "$f" 2>/dev/null | awk -v r="$rocm" 'index($3, r) == 1 || index($3, "/opt/rocm") == 1 {print $3}')
  done
  [ "$added" = 0 ] && break
done
ls "$out"
