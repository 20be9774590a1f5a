"""The API docs generator (reference docs/autogen.py) resolves every documented symbol."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_autogen_renders_all_pages(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "docs"))
    import autogen
    pages = autogen.generate(str(tmp_path / "out"))
    assert len(pages) == len(autogen.PAGES)
    text = open(os.path.join(str(tmp_path / "out"), "api", "models", "spark-model.md")).read()
    assert "class `SparkModel" in text and "fit" in text
    assert os.path.exists(tmp_path / "out" / "index.md")
