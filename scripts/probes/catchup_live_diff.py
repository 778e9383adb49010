"""Debug probe: the first differing catch-up messages between the engine- and oracle-driven live legacy clients."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from fluidframework_amd.engine import Engine  # noqa: E402
from fluidframework_amd.live import EngineExecutor  # noqa: E402
from mock_runtime import OracleExecutor  # noqa: E402
from test_catchup_live import farm_script, replay  # noqa: E402

for seed in (1, 2):
    eng = Engine(4, snapshot_v1=False, max_segments=4096, heap_entries=4096, text_units=1 << 16,
                 prop_words=1 << 14, remover_cells=1 << 12, ref_slots=4096)
    script = farm_script(seed)
    _, mine = replay(EngineExecutor(eng), script)
    _, want = replay(OracleExecutor(legacy=True), script)
    for k, (a, b) in enumerate(zip(mine, want)):
        sa, sb = a.dds.summary(), b.dds.summary()
        print("seed", seed, "client", k, "blobs equal:", [x == y for x, y in zip(sa, sb)], len(sa), len(sb))
        ca, cb = json.loads(sa[-1]), json.loads(sb[-1])
        nd = 0
        for ma, mb in zip(ca, cb):
            if ma != mb:
                nd += 1
                if nd <= 4:
                    print("  engine:", json.dumps(ma))
                    print("  oracle:", json.dumps(mb))
        print("  differing messages:", nd, "of", len(ca), len(cb))
