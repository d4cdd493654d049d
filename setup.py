"""Packaging (replaces distlearn-scm-1.rockspec).

``pip install -e .`` / ``python setup.py build_ext --inplace`` compiles every
HIP/C++ source under csrc/ for gfx950 with hipcc (csrc/build.py) into the
in-tree extension ``torch_distlearn_amd/_C*.so``.
"""
import importlib.util
import os

from setuptools import Command, find_packages, setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


def _native_build():
    spec = importlib.util.spec_from_file_location("_dl_build", os.path.join(ROOT, "csrc", "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.build()


class BuildNative(Command):
    description = "compile the gfx950 HIP kernels + RCCL communicator (hipcc)"
    user_options = []

    def initialize_options(self):
        pass

    def finalize_options(self):
        pass

    def run(self):
        _native_build()


class BuildPy(build_py):
    def run(self):
        _native_build()
        super().run()


setup(
    name="torch_distlearn_amd",
    version="0.1.0",
    description="MI355X-native data-parallel training (AllReduceSGD, AllReduceEA, AsyncEA) with HIP kernels and RCCL",
    license="Apache-2.0",
    packages=find_packages(include=["torch_distlearn_amd", "torch_distlearn_amd.*"]),
    package_data={"torch_distlearn_amd": ["_C*.so"]},
    python_requires=">=3.10",
    install_requires=["torch", "numpy"],
    cmdclass={"build_native": BuildNative, "build_ext": BuildNative, "build_py": BuildPy},
)
