"""HIP (gfx950) kernels of the data plane, built in-tree.

``_dataplane`` is compiled by ``build()`` with hipcc for ``--offload-arch=gfx950``
from csrc/kernels/{engine,dataplane}.hip.  Importing ``chanamq_amd.ops.dataplane``
on a machine with a GPU but without the extension raises: there is no silent
fallback for the hot path.
"""

import importlib
import os
import subprocess
import sys
import sysconfig

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(os.path.dirname(_HERE))
_SRC = os.path.join(_ROOT, "csrc", "kernels")
_EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
EXT_PATH = os.path.join(_HERE, "_dataplane" + _EXT)
SOURCES = ["engine.hip", "dataplane.hip", "dp_state.h", "dp_common.h", "step_abi.h", "xchg_host.h", "xchg_rccl.h"]


def _src_hash():
    import hashlib
    h = hashlib.sha256()
    for s in SOURCES:
        with open(os.path.join(_SRC, s), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _stale():
    """Content-based (mtimes do not survive copies to the GPU box)."""
    if not os.path.exists(EXT_PATH) or not os.path.exists(EXT_PATH + ".srchash"):
        return True
    with open(EXT_PATH + ".srchash") as f:
        return f.read().strip() != _src_hash()


def build(force=False, verbose=False):
    """Compile the data-plane extension for gfx950 (cross-compiles without a GPU)."""
    if not force and not _stale():
        return EXT_PATH
    import pybind11

    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", f"-I{_SRC}"]
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC", *inc,
           os.path.join(_SRC, "engine.hip"), "-o", EXT_PATH + ".tmp", "-L/opt/rocm/lib", "-lhsa-runtime64", "-lrocprofiler-sdk-roctx", "-ldl", "-lrt"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(EXT_PATH + ".tmp", EXT_PATH)
    with open(EXT_PATH + ".srchash", "w") as f:
        f.write(_src_hash())
    return EXT_PATH


def build_variant(path, defines):
    """An A/B build of the same sources with extra -D macros (e.g. ROUTE_WPE=4) at
    ``path``; ``CHANAMQ_DP_SO=path`` makes ``load()`` import it instead."""
    import pybind11

    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", f"-I{_SRC}"]
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC", *inc,
           *[f"-D{d}" for d in defines], os.path.join(_SRC, "engine.hip"), "-o", path + ".tmp",
           "-L/opt/rocm/lib", "-lhsa-runtime64", "-lrocprofiler-sdk-roctx", "-ldl", "-lrt"]
    subprocess.run(cmd, check=True)
    os.replace(path + ".tmp", path)
    return path


STANDIN_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                           "tests", "rccl_standin")
STANDIN_SO = os.path.join(STANDIN_DIR, "librccl_standin.so")


def build_rccl_standin(verbose=False):
    """The tests' shared-memory stand-in for librccl (tests/rccl_standin): lets several
    ranks of the engine's RCCL exchange share one GPU.  Test-only (see ``load``)."""
    src = os.path.join(STANDIN_DIR, "rccl_standin.cpp")
    if not os.path.exists(src):
        return None
    if os.path.exists(STANDIN_SO) and os.path.getmtime(STANDIN_SO) >= os.path.getmtime(src):
        return STANDIN_SO
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "--offload-arch=gfx950", "-O2", "-std=c++17", "-shared", "-fPIC", src, "-o", STANDIN_SO + ".tmp",
           "-lrt"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(STANDIN_SO + ".tmp", STANDIN_SO)
    return STANDIN_SO


def load():
    """Import the compiled extension, rebuilding it first if the sources changed
    (raises ImportError with a build hint if it cannot be built).  Refuses a librccl
    override (CHANAMQ_RCCL_LIB: the tests' stand-in) unless CHANAMQ_RCCL_STANDIN_OK=1 says
    this is a test or a labelled rehearsal."""
    if os.environ.get("CHANAMQ_RCCL_LIB") and os.environ.get("CHANAMQ_RCCL_STANDIN_OK") != "1":
        raise RuntimeError("CHANAMQ_RCCL_LIB names a librccl stand-in: test-only (set CHANAMQ_RCCL_STANDIN_OK=1 "
                           "in tests / labelled rehearsals)")
    alt = os.environ.get("CHANAMQ_DP_SO")
    if alt:   # an A/B variant (build_variant)
        from importlib import util as ilu
        mod = sys.modules.get("chanamq_amd.ops._dataplane")
        if mod is None:
            spec = ilu.spec_from_file_location("chanamq_amd.ops._dataplane", alt)
            mod = ilu.module_from_spec(spec)
            spec.loader.exec_module(mod)
            sys.modules["chanamq_amd.ops._dataplane"] = mod
        return mod
    if _stale():
        build()
    try:
        return importlib.import_module("chanamq_amd.ops._dataplane")
    except ImportError as e:
        raise ImportError(f"chanamq_amd.ops._dataplane is not built ({e}); run "
                          "`python -c 'import __graft_entry__ as g; g.build()'`") from e
