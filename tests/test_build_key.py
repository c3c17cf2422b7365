"""Stale-binary guard: a built module carries the content-hash key of the sources it was linked from
(_build.source_key), and the loader refuses a module whose key does not match the tree."""
import shutil

import pytest

from simple_distributed_machine_learning_amd import _build, _native


def test_modules_carry_the_key_of_the_current_sources():
    _native.runtime()
    for what in ("runtime", "kernels"):
        path = _build.module_path(what)
        if not path.exists():
            pytest.skip(f"{path.name} not built")
        assert _build.embedded_key(path) == _build.source_key(what)


def test_key_follows_every_source_and_header(tmp_path, monkeypatch):
    # a copy of the runtime sources: editing one byte of a header changes the key
    src = tmp_path / "csrc"
    shutil.copytree(_build.CSRC / "runtime", src / "runtime")
    shutil.copytree(_build.CSRC / "common", src / "common")
    monkeypatch.setattr(_build, "CSRC", src)
    k0 = _build.source_key("runtime")
    hdr = sorted((src / "common").glob("*.h"))[0]
    hdr.write_text(hdr.read_text() + "\n// edited\n")
    assert _build.source_key("runtime") != k0


def test_loader_refuses_a_module_built_from_other_sources(tmp_path, monkeypatch):
    path = _build.module_path("runtime")
    if not path.exists():
        pytest.skip("runtime not built")
    fake = tmp_path / path.name
    shutil.copy(path, fake)
    good = _build.source_key("runtime")
    assert _native.check_key(fake, good) == good
    # tampered tree: the sources now hash to another key -> refused
    with pytest.raises(_native.StaleModuleError):
        _native.check_key(fake, "0" * 24)
    # a module from before build keys existed carries no marker -> refused
    data = fake.read_bytes().replace(_build.KEY_MARKER, b"XXXX_BUILD_KEY=")
    fake.write_bytes(data)
    assert _build.embedded_key(fake) is None
    with pytest.raises(_native.StaleModuleError):
        _native.check_key(fake, good)


def test_fresh_refuses_without_autobuild(tmp_path, monkeypatch):
    path = _build.module_path("runtime")
    if not path.exists():
        pytest.skip("runtime not built")
    monkeypatch.setattr(_build, "source_key", lambda what: "f" * 24)
    monkeypatch.setenv("SDML_NO_AUTOBUILD", "1")
    with pytest.raises(_native.StaleModuleError):
        _native._fresh("runtime")
