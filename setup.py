"""Packaging (reference ``setup.py`` packaged only ``megatron.core``; this one
ships the whole framework).  The HIP/C++ extension is built in-tree for gfx950
by ``python -m epfl_megatron_amd.build`` (run it before ``pip install -e .``)."""
from setuptools import find_packages, setup

setup(
    name="epfl_megatron_amd",
    version="0.1.0",
    description="MI355X-native Megatron-LLM (Llama / Llama-2 / Falcon / GPT) training and serving",
    packages=find_packages(include=["epfl_megatron_amd", "epfl_megatron_amd.*", "tasks",
                                    "tasks.*"]),
    package_data={"epfl_megatron_amd": ["csrc/*.h", "csrc/*.hip", "csrc/*.cpp", "*.so",
                                        "inference/static/*.html"]},
    python_requires=">=3.10",
    install_requires=["torch>=2.4", "numpy", "sentencepiece", "regex"],
    extras_require={"convert": ["transformers", "safetensors"],
                    "serve": ["fastapi", "uvicorn"]},
)
