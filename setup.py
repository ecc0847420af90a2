"""Build the in-tree gfx950 extension:  python setup.py build_ext --inplace

Kernels (*.hip) are compiled by hipcc for gfx950 only; the host plan builder and the
pybind11 bindings by the host compiler.  The resulting
network_distributed_pytorch_amd/_C*.so stays in the source tree (it travels to the GPU
box with the snapshot; nothing is installed into site-packages).
"""
import os

import torch
from setuptools import find_packages, setup
from torch.utils.cpp_extension import BuildExtension, CUDAExtension

os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")

CSRC = os.path.join("network_distributed_pytorch_amd", "csrc")
SOURCES = [os.path.join(CSRC, f) for f in ("bindings.cpp", "plan.cpp", "comm.cpp", "powersgd.hip", "orth.hip",
                                                "multitensor.hip", "batchnorm.hip", "attention.hip", "conv.hip",
                                                "pool.hip", "embedding.hip", "linear.hip", "loss.hip", "layernorm.hip",
                                                "tgemm.hip", "ipc.hip", "winograd.hip")]
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _invalidate_on_header_change():
    """hipcc-compiled objects carry no header dependency info for ninja: when a shared header
    changes, drop the object directory so every translation unit is rebuilt (a stale object
    compiled against an old declaration would leave an undefined symbol in _C*.so)."""
    import glob
    import hashlib
    import shutil

    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(CSRC, "*.h"))):
        with open(f, "rb") as fh:
            h.update(fh.read())
    digest = h.hexdigest()
    stamp = os.path.join("build", ".headers.sha256")
    old = open(stamp).read().strip() if os.path.exists(stamp) else None
    if old != digest:
        for d in glob.glob(os.path.join("build", "temp.*")):
            shutil.rmtree(d, ignore_errors=True)
        os.makedirs("build", exist_ok=True)
        with open(stamp, "w") as fh:
            fh.write(digest)


_invalidate_on_header_change()
# RCCL: link the copy torch already loads (SONAME librccl.so.1), so the process holds ONE
# RCCL whether c10d or the native communicator (csrc/comm.cpp) creates a communicator
TORCH_LIB = os.path.join(os.path.dirname(torch.__file__), "lib")

ext = CUDAExtension(
    name="network_distributed_pytorch_amd._C",
    sources=SOURCES,
    include_dirs=[os.path.abspath(CSRC), os.path.join(ROCM, "include")],
    library_dirs=[TORCH_LIB],
    libraries=["rccl"],
    extra_compile_args={
        "cxx": ["-O3", "-std=c++17"],
        "nvcc": ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=fast"],
    },
)

setup(
    name="network_distributed_pytorch_amd",
    version="0.1.0",
    packages=find_packages(include=["network_distributed_pytorch_amd", "network_distributed_pytorch_amd.*"]),
    ext_modules=[ext],
    cmdclass={"build_ext": BuildExtension.with_options(use_ninja=True)},
)
