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


# ---- parameter-cache naming (core/parameter_cache.hpp:50-219) ----
def test_param_cache_identifier_and_paths(tmp_path, monkeypatch):
    """cache_identifier = <cache_prefix>-<hex sha256(identifier)> (:166-171), paths <dir>/v28-<id>.<ext> under
    FIL_PROOFS_PARAMETER_CACHE (:50-56, :78-94), and the reference's PARAMETER_CACHE_DIR when it is unset."""
    import hashlib

    ident = "layered_drgporep::PublicParams{ graph: stacked_graph::StackedGraph{expansion_degree: 8 base_graph: ...}"
    cid = fg.param_cache_id("stacked-proof-of-replication-merkletree-poseidon_hasher-8-8-0-sha256_hasher", ident)
    want = "stacked-proof-of-replication-merkletree-poseidon_hasher-8-8-0-sha256_hasher-" + \
        hashlib.sha256(ident.encode()).hexdigest()
    assert cid == want
    for msg in ["", "a", "x" * 55, "y" * 56, "z" * 64, "w" * 200]:  # SHA-256 padding edges
        assert fg.param_cache_id("p", msg) == "p-" + hashlib.sha256(msg.encode()).hexdigest()
    monkeypatch.setenv("FIL_PROOFS_PARAMETER_CACHE", str(tmp_path))
    assert fg.param_cache_path(cid, fg.PARAMS) == f"{tmp_path}/v28-{cid}.params"
    assert fg.param_cache_path(cid, fg.META) == f"{tmp_path}/v28-{cid}.meta"
    assert fg.param_cache_path(cid, fg.VK) == f"{tmp_path}/v28-{cid}.vk"
    monkeypatch.delenv("FIL_PROOFS_PARAMETER_CACHE")
    assert fg.param_cache_path("x", fg.VK) == "/var/tmp/filecoin-proof-parameters//v28-x.vk"
    with pytest.raises(fg.FilGpuError):
        fg.param_cache_path("x", 3)


def test_param_cache_metadata_read_or_write(tmp_path, monkeypatch):
    """get_param_metadata (:173-183): the first call writes {"sector_size":N}, later calls read it back; a cache
    directory that does not exist is refused (ensure_ancestor_dirs_exist, :96-103)."""
    monkeypatch.setenv("FIL_PROOFS_PARAMETER_CACHE", str(tmp_path))
    cid = fg.param_cache_id("post", "fallback::PublicParams{...}")
    assert fg.param_cache_metadata(cid, 34359738368) == 34359738368
    meta = tmp_path / f"v28-{cid}.meta"
    assert meta.read_text() == '{"sector_size":34359738368}'
    assert fg.param_cache_metadata(cid, 2048) == 34359738368  # cached value wins
    meta.write_text("not json")
    assert fg.param_cache_metadata(cid, 2048) == 2048  # unreadable -> rewritten
    monkeypatch.setenv("FIL_PROOFS_PARAMETER_CACHE", str(tmp_path / "missing"))
    with pytest.raises(fg.FilGpuError) as e:
        fg.param_cache_metadata(cid, 1)
    assert e.value.code == -1 and "no parent directory" in str(e.value)
