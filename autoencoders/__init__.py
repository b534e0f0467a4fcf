"""Alias package giving the reference's pickle module paths (``autoencoders.*``) to the
native classes of ``sparse_coding__amd``."""
