"""Location of committed per-layer tile-config tuning tables (produced on MI355X
by ``python -m kdl.engine.tune``)."""
from __future__ import annotations

from pathlib import Path

TUNING_DIR = Path(__file__).resolve().parent.parent / "tuning"


def tuning_path(model: str, batch: int) -> Path:
    return TUNING_DIR / f"{model}_b{batch}.json"
