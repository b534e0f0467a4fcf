"""Remote-operations helpers (reference ``utils.py`` / ``cmdutil.py``: rsync / scp to a
training host, S3 upload/download of results).

The reference hard-codes a host, user and AWS access keys; here every endpoint comes
from arguments or environment variables (``SC_REMOTE_HOST``, ``SC_REMOTE_PORT``,
``SC_REMOTE_DIR``, ``SC_S3_BUCKET``) and nothing runs at import.  Command builders are
pure functions (testable offline); ``run`` executes one.  S3 needs ``boto3``, which is
optional and absent on this image -- the S3 helpers say so instead of failing obscurely.
"""

from __future__ import annotations

import os
import shlex
import subprocess
from typing import Iterable, List, Optional, Sequence


class dotdict(dict):
    """Attribute access to a dict (reference utils.py:98-119)."""

    __getattr__ = dict.get
    __setattr__ = dict.__setitem__
    __delattr__ = dict.__delitem__


def _host(host: Optional[str]) -> str:
    h = host or os.environ.get("SC_REMOTE_HOST", "")
    if not h:
        raise ValueError("no remote host: pass host= or set SC_REMOTE_HOST")
    return h


def _port(port: Optional[int]) -> int:
    return int(port or os.environ.get("SC_REMOTE_PORT", 22))


def _rdir(remote_dir: Optional[str]) -> str:
    return remote_dir or os.environ.get("SC_REMOTE_DIR", "sparse_coding__amd")


def rsync_push(src: str = ".", host: Optional[str] = None, remote_dir: Optional[str] = None,
               port: Optional[int] = None, include: Sequence[str] = (), exclude: Sequence[str] = (".git",),
               respect_gitignore: bool = True) -> List[str]:
    cmd = ["rsync", "-rv"]
    if respect_gitignore:
        cmd += ["--filter", ":- .gitignore"]
    for p in include:
        cmd += ["--include", p]
    for p in exclude:
        cmd += ["--exclude", p]
    cmd += ["-e", f"ssh -p {_port(port)}", src, f"{_host(host)}:{_rdir(remote_dir)}"]
    return cmd


def rsync_pull(remote_path: str, dst: str, host: Optional[str] = None, port: Optional[int] = None,
               exclude: Sequence[str] = ("*.hdf", "*.pkl")) -> List[str]:
    cmd = ["rsync", "-r"]
    for p in exclude:
        cmd += ["--exclude", p]
    return cmd + ["-e", f"ssh -p {_port(port)}", f"{_host(host)}:{remote_path}", dst]


def scp_push(paths: Iterable[str], host: Optional[str] = None, remote_dir: Optional[str] = None,
             port: Optional[int] = None) -> List[str]:
    return ["scp", "-P", str(_port(port)), "-r", *paths, f"{_host(host)}:{_rdir(remote_dir)}"]


def run(cmd: List[str], dry_run: bool = False) -> int:
    if dry_run:
        print(" ".join(shlex.quote(c) for c in cmd))
        return 0
    return subprocess.call(cmd)


def _s3():
    try:
        import boto3  # optional
    except ImportError as e:
        raise RuntimeError("S3 helpers need boto3, which is not installed on this machine") from e
    return boto3.client("s3")


def upload_to_s3(local_path: str, bucket: Optional[str] = None, prefix: str = "") -> List[str]:
    """Upload a file or a directory tree; returns the object keys written."""
    bucket = bucket or os.environ.get("SC_S3_BUCKET", "")
    if not bucket:
        raise ValueError("no bucket: pass bucket= or set SC_S3_BUCKET")
    client = _s3()
    keys = []
    paths = [local_path] if os.path.isfile(local_path) else [
        os.path.join(r, f) for r, _, fs in os.walk(local_path) for f in fs]
    for p in paths:
        key = os.path.join(prefix, os.path.relpath(p, os.path.dirname(local_path) if os.path.isfile(local_path)
                                                   else os.path.dirname(local_path.rstrip("/"))))
        client.upload_file(p, bucket, key)
        keys.append(key)
    return keys


def download_from_s3(keys: Iterable[str], bucket: Optional[str] = None, dst: str = ".",
                     force: bool = False) -> List[str]:
    bucket = bucket or os.environ.get("SC_S3_BUCKET", "")
    client = _s3()
    out = []
    for k in keys:
        target = os.path.join(dst, k)
        if os.path.exists(target) and not force:
            out.append(target)
            continue
        os.makedirs(os.path.dirname(os.path.abspath(target)), exist_ok=True)
        client.download_file(bucket, k, target)
        out.append(target)
    return out
