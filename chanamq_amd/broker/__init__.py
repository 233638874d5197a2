"""Native broker core (C++): AMQP codec, connection engine, control plane, CPU data path,
embedded Cassandra-schema store.  Built in-tree by ``build()`` with g++ (+OpenSSL)."""

import importlib
import os
import subprocess
import sys
import sysconfig

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(os.path.dirname(_HERE))
_SRC = os.path.join(_ROOT, "csrc", "core")
_EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
EXT_PATH = os.path.join(_HERE, "_core" + _EXT)
SOURCES = ["codec.cpp", "store.cpp", "broker.cpp", "loadgen.cpp", "gateway.cpp", "frontend.cpp", "persist.cpp",
           "bodylog.cpp", "tls_proxy.cpp",            "bindings.cpp"]
HEADERS = ["codec.hpp", "store.hpp", "broker.hpp", "loadgen.hpp", "gateway.hpp", "frontend.hpp", "persist.hpp", "bodylog.hpp", "flatmap.hpp", "tls_proxy.hpp",
           "../kernels/step_abi.h", "../kernels/xchg_host.h"]


def _src_hash():
    import hashlib
    h = hashlib.sha256()
    for s in SOURCES + HEADERS:
        with open(os.path.join(_SRC, s), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _stale():
    """Content-based (mtimes do not survive copies to the GPU box)."""
    if not os.path.exists(EXT_PATH) or not os.path.exists(EXT_PATH + ".srchash"):
        return True
    with open(EXT_PATH + ".srchash") as f:
        return f.read().strip() != _src_hash()


def build(force=False, verbose=False, sanitize=None):
    """g++ -O2 shared library; ``sanitize='address'|'thread'`` builds an instrumented
    copy for host-side race/memory checks."""
    if not force and not sanitize and not _stale():
        return EXT_PATH
    import pybind11

    cxx = os.environ.get("CXX", "g++")
    out = EXT_PATH if not sanitize else EXT_PATH.replace("_core", f"_core_{sanitize}")
    flags = ["-O2", "-g", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wno-unused-result"]
    if sanitize:
        flags += [f"-fsanitize={sanitize}", "-fno-omit-frame-pointer"]
    cmd = [cxx, *flags, f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
           *[os.path.join(_SRC, s) for s in SOURCES], "-o", out + ".tmp", "-lssl", "-lcrypto", "-lpthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    if not sanitize:
        with open(out + ".srchash", "w") as f:
            f.write(_src_hash())
    return out


def load():
    if _stale():
        build()
    try:
        return importlib.import_module("chanamq_amd.broker._core")
    except ImportError as e:
        raise ImportError(f"chanamq_amd.broker._core is not built ({e}); run __graft_entry__.build()") from e
