"""CosmoMC ``.ini`` reader (subset of TIniFile, reference source/IniObjects.f90).

key = value lines, ``#`` comments, ``INCLUDE(file)`` / ``DEFAULT(file)``
(first definition wins, IniObjects.f90:426-490), ``%DATASETDIR%`` /
``%LOCALDIR%`` substitution (settings.f90:183-184), relative file names
resolved against the including file (ResolveLinkedFile, :403-424).
"""
from __future__ import annotations

import os


class IniFile:
    def __init__(self, filename: str | None = None, text: str | None = None,
                 datasetdir: str | None = None):
        self._kv: dict[str, str] = {}
        self._origin: dict[str, str] = {}
        self.filename = filename or ""
        self.datasetdir = datasetdir or os.environ.get("COSMOMC_DATASETDIR", "data/")
        if filename:
            self._open(filename, 0)
        if text:
            self._parse_lines(text.splitlines(), self.filename or os.getcwd() + "/", 0)

    def _parse_lines(self, lines, fname, depth):
        includes, defaults = [], []
        for raw in lines:
            t = raw.strip()
            if t == "END":
                break
            if not t or t.startswith("#"):
                continue
            if t.startswith("INCLUDE(") or t.startswith("DEFAULT("):
                close = t.find(")")
                if close < 0:
                    raise ValueError(f"bad include line in {fname}: {t}")
                (includes if t[0] == "I" else defaults).append(t[8:close])
                continue
            if "=" not in t:
                continue
            k, v = t.split("=", 1)
            k, v = k.strip(), v.strip()
            if k and k not in self._kv:
                self._kv[k] = v
                self._origin[k] = fname
        for f in includes + defaults:
            self._open(self._resolve_linked(f, fname), depth + 1)

    def _open(self, filename, depth):
        if depth > 16:
            raise ValueError("INCLUDE/DEFAULT nesting too deep")
        with open(filename) as f:
            self._parse_lines(f.read().splitlines(), filename, depth)

    @staticmethod
    def _resolve_linked(name, thisfile):
        if os.path.isabs(name):
            return name
        cand = os.path.join(os.path.dirname(thisfile), name)
        return cand if os.path.exists(cand) else name

    def keys(self):
        return list(self._kv.keys())

    def __contains__(self, k):
        return k in self._kv

    def __getitem__(self, k):
        return self._kv[k]

    def get(self, k, default=None):
        return self._kv.get(k, default)

    def set(self, k, v):
        self._kv[k] = str(v)

    def read_int(self, k, default=None):
        v = self._kv.get(k)
        return default if v in (None, "") else int(v)

    def read_float(self, k, default=None):
        v = self._kv.get(k)
        return default if v in (None, "") else float(v)

    def read_bool(self, k, default=False):
        v = self._kv.get(k)
        if v in (None, ""):
            return default
        return v.strip().upper() in ("T", "TRUE", ".TRUE.", "1", "Y", "YES")

    def resolve(self, value: str, origin: str | None = None) -> str:
        v = value.replace("%DATASETDIR%", self.datasetdir).replace("%LOCALDIR%", "./")
        if os.path.isabs(v):
            return v
        base = origin or self.filename
        cand = os.path.join(os.path.dirname(base), v) if base else v
        return cand if os.path.exists(cand) else v

    def relative_filename(self, k: str) -> str:
        return self.resolve(self._kv[k], self._origin.get(k))
