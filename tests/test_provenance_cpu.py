"""Binary provenance of the kernel library: the sha256 of the kernel sources is compiled into
``_sc_kernels.so`` and the loader refuses a library built from other sources."""
import pytest

from sparse_coding__amd.ops import _lib, build


def test_source_hash_is_stable_and_content_based(tmp_path, monkeypatch):
    h = build.source_hash()
    assert len(h) == 64 and h == build.source_hash()
    # a change in any source changes the identity
    fake = tmp_path / "csrc"
    fake.mkdir()
    (fake / "a.hip").write_text("kernel one")
    monkeypatch.setattr(build, "CSRC", fake)
    h1 = build.source_hash()
    (fake / "a.hip").write_text("kernel two")
    assert build.source_hash() != h1


def test_shipped_library_matches_tree():
    if not build.LIB.exists():
        pytest.skip("kernel library not built in this tree")
    assert build.embedded_hash() == build.source_hash(), "stale _sc_kernels.so: rebuild it"
    assert _lib.verify_provenance() == build.source_hash()


def test_library_from_other_sources_is_refused(tmp_path):
    if not build.LIB.exists():
        pytest.skip("kernel library not built in this tree")
    data = bytearray(build.LIB.read_bytes())
    i = data.find(build.HASH_TAG) + len(build.HASH_TAG)
    data[i:i + 64] = b"0" * 64  # a library built from different sources
    bad = tmp_path / "_sc_kernels.so"
    bad.write_bytes(bytes(data))
    with pytest.raises(_lib.KernelError, match="different kernel sources"):
        _lib.verify_provenance(bad)
    untagged = tmp_path / "untagged.so"
    untagged.write_bytes(b"\x7fELF no tag")
    with pytest.raises(_lib.KernelError, match="untagged"):
        _lib.verify_provenance(untagged)
