"""Versioned model repository: latest-version policy and hot swap (CPU backend)."""
import json

import pytest

from kdl.serving.config import BatchingParams, ServerConfig
from kdl.serving.model_repo import AVAILABLE, END, ModelManager, list_versions

pytest.importorskip("kdl._rt")


def _cfg(base):
    return ServerConfig(port=0, rest_api_port=0, model_base_path=str(base), device="cpu",
                        file_system_poll_wait_seconds=0,
                        batching=BatchingParams(max_batch_size=2, allowed_batch_sizes=[1, 2]))


def test_latest_version_and_hot_swap(tmp_path):
    base = tmp_path / "clothing-model"
    (base / "1").mkdir(parents=True)
    (base / "1" / "synthetic.json").write_text(json.dumps({"seed": 1}))
    (base / "notaversion").mkdir()
    m = ModelManager(_cfg(base))
    m.load_initial()
    assert m.get("clothing-model").version == 1
    (base / "3").mkdir()
    (base / "3" / "synthetic.json").write_text(json.dumps({"seed": 3}))
    assert list_versions(base) == [1, 3]
    m.reload()
    assert m.get("clothing-model").version == 3
    st = {v: s for v, s, _ in m.status()}
    assert st == {1: END, 3: AVAILABLE}
    m.close()


def test_empty_repo_requires_synthetic(tmp_path):
    with pytest.raises(FileNotFoundError):
        ModelManager(_cfg(tmp_path / "none")).load_initial()
