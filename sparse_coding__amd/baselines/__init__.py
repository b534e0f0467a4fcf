"""Baseline dictionaries: PCA (streaming, GPU), ICA / NMF (scikit-learn), random / identity
(``models.learned_dict``) and the layer sweep that matches their sparsity to learned dicts."""
