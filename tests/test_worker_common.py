"""Worker-side helpers (kubedl_amd/workers/common.py)."""
import json

from kubedl_amd.workers import common


def test_progress_writes_are_throttled_but_first_and_final_land(tmp_path, monkeypatch):
    path = tmp_path / "progress.0"
    monkeypatch.setenv("KDL_PROGRESS_FILE", str(path))
    monkeypatch.setenv("KDL_TUNE", "progress_min_s=30")
    monkeypatch.setattr(common, "_PROGRESS_LAST", [0.0])
    common.report_progress(1)
    assert json.loads(path.read_text())["step"] == 1
    for s in range(2, 50):  # inside the window: no write (the host cost of a file per step)
        common.report_progress(s)
    assert json.loads(path.read_text())["step"] == 1
    common.report_progress(50, final=True)
    assert json.loads(path.read_text())["step"] == 50


def test_progress_every_step_without_throttle(tmp_path, monkeypatch):
    path = tmp_path / "progress.0"
    monkeypatch.setenv("KDL_PROGRESS_FILE", str(path))
    monkeypatch.setenv("KDL_TUNE", "progress_min_s=0")
    monkeypatch.setattr(common, "_PROGRESS_LAST", [0.0])
    for s in range(1, 4):
        common.report_progress(s, 2.5)
        d = json.loads(path.read_text())
        assert d["step"] == s and d["steps_per_sec"] == 2.5
