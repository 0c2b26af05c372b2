"""metaopt_amd -- an MI355X-native meta-optimization (hyper-parameter search) framework.

Host control plane: search spaces and priors, algorithms (random, ASHA, TPE, PBT, ...),
experiments and trials in a document store, asynchronous workers, experiment version control and
the ``mopt`` CLI.  Device data plane: populations of trials trained side by side on gfx950 with
hand-written HIP kernels, sharded one process per GPU over RCCL.
"""
__version__ = "0.2.0"
