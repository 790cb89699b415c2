"""Evidence hygiene: every committed profiles/*.json parses
as one JSON document."""
import json
import pathlib

ROOT = pathlib.Path(__file__).resolve().parent.parent


def test_every_profile_json_parses():
    files = sorted((ROOT / "profiles").rglob("*.json"))
    assert files
    bad = []
    for f in files:
        try:
            json.loads(f.read_text())
        except ValueError as e:
            bad.append(f"{f.relative_to(ROOT)}: {e}")
    assert not bad, bad
