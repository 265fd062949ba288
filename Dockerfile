# Multi-stage image for every component (reference Dockerfile:1-28 shipped
# /app/{admission,controller,synchronizer}; this one adds the MI355X node agent, crdgen,
# kube-lite and the gfx950 diagnostics library).
ARG ROCM_IMAGE=rocm/dev-ubuntu-22.04:7.2

FROM ${ROCM_IMAGE} AS build
RUN apt-get update && apt-get install -y --no-install-recommends \
      cmake ninja-build g++ libssl-dev python3-dev python3-pip && \
    pip3 install pybind11 && rm -rf /var/lib/apt/lists/*
WORKDIR /src
COPY CMakeLists.txt ./
COPY native ./native
RUN cmake -S . -B build -G Ninja -DCMAKE_BUILD_TYPE=Release && \
    ninja -C build crdgen controller admission synchronizer node-agent kube-lite bgc-certgen && \
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared \
      -mllvm -amdgpu-mfma-vgpr-form=1 -Inative/gpu/hip native/gpu/hip/gpu_diag.hip \
      -o bin/libbgc_gpu_diag.so

# Runtime: ROCm user-space (HIP runtime + libamd_smi) for the node agent; the control
# plane binaries only need libssl.
FROM ${ROCM_IMAGE} AS runtime
RUN apt-get update && apt-get install -y --no-install-recommends ca-certificates libssl3 && \
    rm -rf /var/lib/apt/lists/*
COPY --from=build /src/bin/ /app/
# GLIBC_TUNABLES: deeper malloc tcache (+14% CR/s measured, profiles/malloc_tunables_r1/)
ENV BGC_GPU_DIAG_LIB=/app/libbgc_gpu_diag.so \
    LD_LIBRARY_PATH=/opt/rocm/lib \
    GLIBC_TUNABLES=glibc.malloc.tcache_count=64:glibc.malloc.tcache_max=16384
USER 65532:65532
