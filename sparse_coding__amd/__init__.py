"""sparse_coding__amd: an MI355X-native sparse-dictionary-learning engine.

Capabilities of johnathan217/sparse_coding_ (ensembles of sparse autoencoders
over L1 sweeps, tied/untied/masked/top-k/FISTA dictionary learners, the
LearnedDict API and its checkpoint format, activation harvesting, metrics and
baselines), rebuilt around hand-written gfx950 HIP kernels, HBM-resident
activation rings and RCCL over xGMI.
"""

__version__ = "0.1.0"
