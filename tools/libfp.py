"""Fingerprints of the product library for tying PMC counters to the build they were
collected on: the binary's sha256, and the sha256 of the sources and build script it is
compiled from. hipcc's output is not byte-reproducible (the code object's symbol table
order varies between builds of the same source), so a rebuild of unchanged sources — as
the round-end build step does — keeps the source fingerprint while the binary one moves."""
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = [("pm-rl_amd", "csrc"), ("include",)]
BUILD = os.path.join("pm-rl_amd", "build.py")


def file_sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def source_sha256(root=ROOT):
    """sha256 over (relative path, contents) of every file the product library is built
    from (pm-rl_amd/csrc/*, include/*) and the build script; None when they are absent."""
    files = [BUILD]
    for parts in SOURCES:
        d = os.path.join(root, *parts)
        if not os.path.isdir(d):
            return None
        files += [os.path.join(*parts, f) for f in sorted(os.listdir(d)) if os.path.isfile(os.path.join(d, f))]
    h = hashlib.sha256()
    for rel in files:
        p = os.path.join(root, rel)
        if not os.path.exists(p):
            return None
        h.update(rel.encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()
