"""tools/shape_baseline.py's comparison (CPU): a shape slower than the table by more than the tolerance is flagged,
faster or within-tolerance shapes are not, shapes missing from the new run are reported, and the committed table
covers every study model's five batch-1 GEMM roles on MXFP4 and Q4_K."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))

import shape_baseline  # noqa: E402


def test_compare_flags_only_regressions_beyond_tolerance():
    table = {"m/fp4/o": 5.0, "m/fp4/qkv": 8.0, "m/fp4/down": 9.0, "m/fp4/lm_head": 50.0}
    now = {"m/fp4/o": 5.3, "m/fp4/qkv": 8.8, "m/fp4/down": 7.0}
    rows = {r["shape"]: r for r in shape_baseline.compare(table, now, 0.08)}
    assert not rows["m/fp4/o"]["regressed"] and rows["m/fp4/o"]["ratio"] == 1.06
    assert rows["m/fp4/qkv"]["regressed"]
    assert not rows["m/fp4/down"]["regressed"]
    assert rows["m/fp4/lm_head"]["missing"] and not rows["m/fp4/lm_head"]["regressed"]


def test_committed_table_covers_the_study_models():
    path = ROOT / "baselines" / "b1_shapes_mi355x.json"
    doc = json.loads(path.read_text())
    shapes = doc["shapes"]
    for m in shape_baseline.MODELS:
        for dt in shape_baseline.DTYPES.split(","):
            for role in shape_baseline.ROLES.split(","):
                k = f"{m}/{dt}/{role}"
                assert k in shapes and 0.5 < shapes[k] < 1000.0, k
