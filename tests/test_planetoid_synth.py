"""The synthetic Planetoid writer is deterministic (the GPU e2e test relies on
regenerating exactly the dataset the reference was run on)."""
import hashlib
import os

from planetoid_synth import write_planetoid


def _digest(d):
    h = hashlib.sha256()
    for name in sorted(os.listdir(os.path.join(d, "data"))):
        with open(os.path.join(d, "data", name), "rb") as f:
            h.update(name.encode() + f.read())
    return h.hexdigest()


def test_writer_is_deterministic(tmp_path):
    a, b = tmp_path / "a", tmp_path / "b"
    write_planetoid(str(a))
    write_planetoid(str(b))
    assert _digest(str(a)) == _digest(str(b))
