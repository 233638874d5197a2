"""Builds the two in-tree extensions before packaging: the HIP data plane (hipcc,
--offload-arch=gfx950) and the native broker core (g++ + OpenSSL)."""

from setuptools import setup
from setuptools.command.build_py import build_py


class BuildExtensions(build_py):
    def run(self):
        from chanamq_amd import broker, ops
        ops.build(verbose=True)
        broker.build(verbose=True)
        super().run()


setup(cmdclass={"build_py": BuildExtensions})
