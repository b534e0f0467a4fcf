"""Harvest activation chunks for one or more layers (reference ``generate_test_data.py``).

    python -m sparse_coding__amd.data.generate_test_data --model pythia-70m --layers 2,3 \
        --dataset_folder activation_data --n_chunks 1 --chunk_size_gb 0.5

Writes ``{dataset_folder}/{layer_folder_fmt}/{i}.pt`` fp16 chunks with one forward
per batch for all layers.  Tokens are a synthetic Zipf stream unless ``--token_file``
names a ``.pt`` LongTensor ``[N, seq]`` (or ``--text_file`` + ``--tokenizer_dir``
name local text and a local tokenizer); the LM is random-init unless
``--pretrained_dir`` holds a local HF checkpoint (no network on this machine).
"""

from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List

import torch

from ..utils.config import BaseArgs, _default_device
from . import harvest


@dataclass
class GenTestArgs(BaseArgs):
    model: str = "pythia-70m"
    n_chunks: int = 1
    skip_chunks: int = 0
    chunk_size_gb: float = 2.0
    layers: List[int] = field(default_factory=lambda: [2])
    location: str = "residual"
    dataset_folder: str = "activation_data"
    layer_folder_fmt: str = "layer_{layer}"
    device: str = field(default_factory=_default_device)
    batch_size: int = 64
    seq_len: int = 256
    seed: int = 0
    token_file: str = ""
    text_file: str = ""
    tokenizer_dir: str = ""
    pretrained_dir: str = ""


def _token_batches(args: GenTestArgs):
    if args.token_file:
        toks = torch.load(args.token_file, weights_only=True)
    elif args.text_file:
        import transformers

        tok = transformers.AutoTokenizer.from_pretrained(args.tokenizer_dir)
        with open(args.text_file) as fh:
            toks = harvest.chunk_and_tokenize(fh.read().split("\n\n"), tok, args.seq_len)
    else:
        return harvest.synthetic_token_batches(harvest._dims(args.model)["vocab"], args.batch_size, args.seq_len,
                                               seed=args.seed)

    def gen():
        while True:  # cycle over the file's rows
            for i in range(0, toks.shape[0] - args.batch_size + 1, args.batch_size):
                yield toks[i:i + args.batch_size]

    return gen()


def main(argv=None):
    args = GenTestArgs.from_cli(argv)
    folders = [os.path.join(args.dataset_folder, args.layer_folder_fmt.format(layer=L)) for L in args.layers]
    for f in folders:
        os.makedirs(f, exist_ok=True)
    model = harvest.build_model(args.model, device=args.device, seed=args.seed, pretrained_dir=args.pretrained_dir)
    rows = harvest.setup_data(args.model, folders, list(args.layers), args.location, n_chunks=args.n_chunks,
                              chunk_size_gb=args.chunk_size_gb, device=args.device, skip_chunks=args.skip_chunks,
                              batch_size=args.batch_size, seq_len=args.seq_len, token_batches=_token_batches(args),
                              seed=args.seed, model=model)
    print(f"wrote {rows} rows per layer into {folders}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
