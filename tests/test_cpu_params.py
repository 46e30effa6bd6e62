"""CPU: the params-file header walk of mi_params_inspect (bellman Parameters::write layout of
filecoin v28-*.params files) on keys exported by the oracle, and rejection of malformed files.
No device is needed for inspection."""
import pytest

import circuits
import fil_groth16 as fg
import params_io


@pytest.fixture(scope="module")
def exported(oracle):
    n_in, n_aux, rows, z = circuits.random_circuit(11, 24)
    oc = oracle.OracleCircuit(len(rows), n_in, n_aux, circuits.to_csr(rows))
    return oracle.OracleParams(oc, circuits.toxic()).export()


def test_inspect_counts(tmp_path, exported):
    p = tmp_path / "v28-test.params"
    p.write_bytes(params_io.params_bytes(exported))
    got = fg.params_inspect(str(p))
    want = {"ic": len(exported["ic"]) // 96, "h": len(exported["h"]) // 96, "l": len(exported["l"]) // 96,
            "a": len(exported["a"]) // 96, "b_g1": len(exported["b_g1"]) // 96,
            "b_g2": len(exported["b_g2"]) // 192}
    assert got == want


@pytest.mark.parametrize("cut", [0, 10, 863, 864 + 3, -1, -192])
def test_inspect_rejects_truncated(tmp_path, exported, cut):
    data = params_io.params_bytes(exported)
    p = tmp_path / "bad.params"
    p.write_bytes(data[:cut] if cut >= 0 else data[:len(data) + cut])
    with pytest.raises(fg.FilGpuError) as e:
        fg.params_inspect(str(p))
    assert e.value.code == -1 and "truncated" in str(e.value)  # MI_ERR_ARG


def test_inspect_rejects_trailing_and_missing(tmp_path, exported):
    p = tmp_path / "trail.params"
    p.write_bytes(params_io.params_bytes(exported) + b"\0")
    with pytest.raises(fg.FilGpuError, match="trailing"):
        fg.params_inspect(str(p))
    with pytest.raises(fg.FilGpuError, match="cannot open"):
        fg.params_inspect(str(tmp_path / "missing.params"))
