"""The HIP extension imports on a machine without a GPU (the build check), through the
same ``ops.load()`` every GPU path uses."""


def test_ops_load_imports_the_engine_module():
    from chanamq_amd import ops
    m = ops.load()
    assert hasattr(m, "Engine")
