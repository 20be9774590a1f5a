"""Build shim: ``pip install .`` / ``python setup.py build_ext --inplace`` compile the
native runtime (csrc/, hipcc --offload-arch=gfx950) into elephas_amd/_C*.so via
elephas_amd/_build.py, the same in-tree build ``__graft_entry__.build()`` runs."""
import os
import sys

from setuptools import setup
from setuptools.command.build_py import build_py
from setuptools.command.build_ext import build_ext

ROOT = os.path.dirname(os.path.abspath(__file__))


def _native():
    sys.path.insert(0, ROOT)
    from elephas_amd import _build
    return _build.build(verbose=True)


class BuildNative(build_ext):
    def run(self):
        _native()


class BuildPy(build_py):
    def run(self):
        if os.environ.get("ELEPHAS_AMD_SKIP_NATIVE") != "1":
            _native()
        super().run()


setup(cmdclass={"build_ext": BuildNative, "build_py": BuildPy})
