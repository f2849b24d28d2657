"""Package metadata and build hook: ``build_py`` first compiles the gfx950 HIP kernels (_C) and the
C++ serving runtime (_rt) in-tree with ``nv_genai_amd._build`` (hipcc --offload-arch=gfx950 /
g++), then packages them with the Python sources.

    pip install --no-build-isolation .        # offline: uses the torch/pybind11 already installed
"""
import os
import sys

from setuptools import Distribution, find_packages, setup

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from setuptools.command.build_py import build_py


class BuildNative(build_py):
    def run(self):
        from nv_genai_amd import _build

        _build.build_all()
        super().run()


class NativeDistribution(Distribution):
    """The wheel carries compiled gfx950 / host extensions: tag it per platform."""

    def has_ext_modules(self):
        return True


setup(
    distclass=NativeDistribution,
    name="nv_genai_amd",
    version="0.1.0",
    description="MI355X-native RAG serving framework: gfx950 HIP kernels, C++ serving runtime, RCCL over xGMI",
    python_requires=">=3.10",
    packages=find_packages(include=["nv_genai_amd", "nv_genai_amd.*"]),
    package_data={"nv_genai_amd": ["*.so", "assets/*", "assets/*/*", "csrc/*", "csrc/*/*"]},
    install_requires=["torch", "numpy", "fastapi", "uvicorn", "pydantic>=2", "tokenizers", "safetensors",
                      "jinja2", "requests", "httpx", "aiohttp", "pyyaml"],
    extras_require={"test": ["pytest", "pytest-timeout", "hypothesis"]},
    entry_points={"console_scripts": [
        "nga-model-server = nv_genai_amd.serving.model_server:main",
        "nga-tp-server = nv_genai_amd.serving.tp_server:main",
        "nga-router = nv_genai_amd.serving.router:main",
        "nga-frontend = nv_genai_amd.frontend.__main__:main",
        "nga-sft = nv_genai_amd.training.sft:main",
        "nga-pretrain = nv_genai_amd.training.pretrain:main",
        "nga-evaluate = nv_genai_amd.tools.evaluation.__main__:main",
        "nga-ingest = nv_genai_amd.ingest.streaming:main",
        "nga-doctor = nv_genai_amd.tools.doctor:main",
    ]},
    cmdclass={"build_py": BuildNative},
)
