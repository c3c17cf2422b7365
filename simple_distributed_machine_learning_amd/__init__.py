"""simple_distributed_machine_learning_amd — an MI355X-native split-model (pipeline-parallel)
training engine with the capabilities of maduc238/simple_distributed_machine_learning.

Layers (see SURVEY.md §1 for the reference's layer map):

* ``cli`` / ``train``       — reference-compatible launcher + train/test driver
* ``parallel``              — mesh (RCCL/Gloo process groups), p2p transport, schedules, engine
* ``models``                — stage builders (ref CNN, MLPs, ResNet-18-style, GPT-2)
* ``ops``                   — fused gfx950 HIP kernels (+ PyTorch references for CPU)
* ``data``                  — on-device synthetic MNIST-shape / token datasets
* ``utils``                 — flat buffers, checkpoints, metrics, timers, failure detection
"""
__version__ = "0.1.0"
