"""Location of committed per-layer tile-config tuning tables (produced on MI355X
by ``python -m kdl.engine.tune``)."""
from __future__ import annotations

from pathlib import Path

TUNING_DIR = Path(__file__).resolve().parent.parent / "tuning"


def tuning_path(model: str, batch: int, lanes: int = 1) -> Path:
    """``lanes > 1``: the table tuned with the lanes running concurrently
    (kdl/engine/lanes.py); callers fall back to the single-lane table if absent."""
    return TUNING_DIR / (f"{model}_b{batch}.json" if lanes == 1 else f"{model}_b{batch}_l{lanes}.json")
