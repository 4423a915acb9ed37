"""The zbackup-side binding (integration/gpu_backup_creator.hh) compiles
against include/zchunk.h: the zutils.cc loops of tests/adapter/adapter_main.cpp
over the adapter, built with -Wall -Werror and linked to libzchunk.so (CPU
only: nothing runs on a GPU here)."""
import os

import pytest

from tests.adapter import build as adapter_build


def test_adapter_compiles_and_links(tmp_path):
    from zbackup_amd import _build
    _build.build()
    out = adapter_build.build(str(tmp_path / "adapter_main"))
    assert os.path.getsize(out) > 0
