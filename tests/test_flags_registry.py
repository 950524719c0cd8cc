"""Every BFLY_* environment variable the framework reads — from Python or from the kernel /
runtime libraries (getenv) — is registered in utils/flags.py, so `python -m butterfly_amd
info` lists it with its default and meaning."""
import pathlib
import re

from butterfly_amd.utils import flags

ROOT = pathlib.Path(__file__).resolve().parents[1]
PAT = re.compile(r'getenv\("(BFLY_[A-Z0-9_]+)"\)|environ(?:\.get)?\(?\[?"(BFLY_[A-Z0-9_]+)"|'
                 r'(?:flags\.get|setdefault)\("(BFLY_[A-Z0-9_]+)"')


def test_every_read_env_flag_is_registered():
    used = {}
    files = [p for d in ("csrc", "butterfly_amd") for p in (ROOT / d).rglob("*")
             if p.suffix in (".hip", ".cpp", ".h", ".inc", ".py")] + [ROOT / "bench.py"]
    for p in files:
        for m in PAT.finditer(p.read_text()):
            name = next(g for g in m.groups() if g)
            used.setdefault(name, []).append(str(p.relative_to(ROOT)))
    missing = {k: v for k, v in used.items() if k not in flags.FLAGS}
    assert not missing, f"unregistered flags: {missing}"
    assert len(used) > 40
