"""Package metadata. The HIP extension is built in-tree by ``python -m llm_training_amd._build``
(hipcc, gfx950) — see __graft_entry__.build()."""
from setuptools import find_packages, setup

setup(
    name="llm-training-amd",
    version="0.1.0",
    description="MI355X-native LLM training framework (HIP kernels, RCCL, ZeRO + TP/SP)",
    packages=find_packages(include=["llm_training_amd", "llm_training_amd.*"]),
    package_data={"llm_training_amd": ["csrc/*.hip", "csrc/*.h", "csrc/*.cpp", "_C.so",
                                       "data/chat_templates/*.j2"]},
    python_requires=">=3.10",
    install_requires=["torch", "pydantic>=2", "pyyaml", "safetensors", "transformers", "datasets", "jinja2"],
    entry_points={"console_scripts": ["llm-training = llm_training_amd.cli.main:main"]},
)
