"""Pin the CPU oracle against the reference's own golden vectors."""
import os

import pytest

from fixtures import (SNAPSHOT_VERSIONS, blob_names, load_replay, load_snapshots, replay_files,
                      replay_log, snapshot_log)
from fluidframework_amd.batch import Interner, build_batch
from oracle.oracle import OracleDoc, options


@pytest.mark.parametrize("path", replay_files(), ids=lambda p: os.path.basename(p)[:-8])
def test_replay_text_after_every_group(path):
    """client.replay.spec.ts:17-71 -- text after every group equals resultText."""
    groups = load_replay(path)
    it = Interner()
    log = replay_log(groups, it)
    doc = OracleDoc(options())
    assert doc.apply(build_batch([log], it), 0) == 0
    for gi, g in enumerate(groups):
        assert doc.text() == g["initialText"], f"group {gi} initial"
        for m in g["msgs"]:
            log.message(m, it)
        assert doc.apply(build_batch([log], it), 0) == 0
        assert doc.text() == g["resultText"], f"group {gi}"


SNAPS = load_snapshots()


@pytest.mark.parametrize("key", sorted(SNAPS))
def test_snapshot_blobs_byte_exact(key):
    """generateSharedStrings.ts recipes -> content/ blobs byte-for-byte (snapshotVersion.spec.ts:137-160)."""
    version, name = key.split("/")
    v1 = SNAPSHOT_VERSIONS[version]
    it = Interner()
    log = snapshot_log(name, it)
    b = build_batch([log], it)
    doc = OracleDoc(options(snapshot_v1=v1))
    assert doc.apply(b, 0) == 0
    blobs = doc.summarize(b, 0)
    got = dict(zip(blob_names(len(blobs), v1), blobs))
    exp = {k: v.encode("utf-8") for k, v in SNAPS[key].items()}
    assert got == exp
