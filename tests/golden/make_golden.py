"""Convert the reference's committed golden vectors into compact fixtures under tests/golden/.

Run in the build container (the only place /root/reference exists):
    python tests/golden/make_golden.py

Sources (data files only; no reference source text is copied):
  * packages/dds/merge-tree/src/test/results/*.json  -- 30 replay logs (ReplayGroup[],
    mergeTreeOperationRunner.ts:191-196) replayed by client.replay.spec.ts:17-71.
    Kept fields: initialText, resultText and per message clientId, sequenceNumber,
    referenceSequenceNumber, minimumSequenceNumber, type, contents.
  * packages/dds/sequence/src/test/snapshots/*/*.json -- ITree summaries compared by
    snapshotVersion.spec.ts:137-160.  Kept: the `content` subtree's blob contents (the merge-tree
    summary) -> snapshots.json.gz, and the top-level `header` blob (the interval collections, present in
    the four withIntervals / withV1Intervals files) -> interval_headers.json.
"""
import glob
import gzip
import json
import os

REF = "/root/reference/packages/dds"
HERE = os.path.dirname(os.path.abspath(__file__))


def replay():
    out_dir = os.path.join(HERE, "replay")
    os.makedirs(out_dir, exist_ok=True)
    for f in sorted(glob.glob(f"{REF}/merge-tree/src/test/results/*.json")):
        groups = json.load(open(f))
        slim = []
        for g in groups:
            slim.append(
                {
                    "initialText": g["initialText"],
                    "resultText": g["resultText"],
                    "msgs": [
                        {
                            k: m[k]
                            for k in (
                                "clientId",
                                "sequenceNumber",
                                "referenceSequenceNumber",
                                "minimumSequenceNumber",
                                "type",
                                "contents",
                            )
                        }
                        for m in g["msgs"]
                    ],
                }
            )
        name = os.path.basename(f).replace(".json", ".json.gz")
        with gzip.open(os.path.join(out_dir, name), "wt", encoding="utf-8") as fh:
            json.dump(slim, fh, separators=(",", ":"))


def snapshots():
    res = {}
    for f in sorted(glob.glob(f"{REF}/sequence/src/test/snapshots/*/*.json")):
        tree = json.load(open(f))
        version = os.path.basename(os.path.dirname(f))
        name = os.path.basename(f)[:-5]
        content = [e for e in tree["entries"] if e["path"] == "content"][0]["value"]["entries"]
        res[f"{version}/{name}"] = {b["path"]: b["value"]["contents"] for b in content}
    with gzip.open(os.path.join(HERE, "snapshots.json.gz"), "wt", encoding="utf-8") as fh:
        json.dump(res, fh, separators=(",", ":"))


def interval_headers():
    res = {}
    for f in sorted(glob.glob(f"{REF}/sequence/src/test/snapshots/*/*.json")):
        tree = json.load(open(f))
        h = [e for e in tree["entries"] if e["path"] == "header"]
        if h:
            res[f"{os.path.basename(os.path.dirname(f))}/{os.path.basename(f)[:-5]}"] = h[0]["value"]["contents"]
    with open(os.path.join(HERE, "interval_headers.json"), "w", encoding="utf-8") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    replay()
    snapshots()
    interval_headers()
