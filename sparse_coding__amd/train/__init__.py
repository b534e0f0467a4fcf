"""Training drivers: sweep orchestration, the experiment catalogue and CLIs."""
