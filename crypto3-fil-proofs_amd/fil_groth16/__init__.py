"""fil_groth16 -- MI355X-native Groth16 proving core (BLS12-381) for Filecoin Seal / PoSt.

Host-side mirror of the reference's prover interface over libfilgpu.so's C ABI
(include/mi355x_groth16.h).  See DESIGN.md for the hot path and INTEGRATION.md for the
reference-side binding.
"""
from ._lib import EXPORTS, LIB_PATH, FilGpuError, build, lib  # noqa: F401
from .core import (FR_MODULUS, PROOF_BYTES, SHARE_BYTES, VK_BYTES, Circuit, Context, HostBuffer, Points,  # noqa: F401
                   ProvingKey, assemble, device_count, fr_bytes, generate_random_parameters, msm_window_bits,
                   params_inspect, pairing, prove, param_cache_id, param_cache_path, param_cache_metadata,
                   get_groth_params, PARAMS, META, VK, prove_batch, prove_share, prove_share_ranges, h_coeffs_dev, trapdoor_dlogs, verify, verify_batch)
from .compound import (MultiProof, partition_count, get_partitions_for_window_post,  # noqa: F401
                       circuit_proofs, seal_commit_phase2_proofs, generate_window_post_proofs,
                       generate_winning_post_proof, select_challenges, porep_layer_challenges, LayerChallenges)
from . import tree  # noqa: F401  (Poseidon + tree C / tree R-last builders)
from . import stacked  # noqa: F401  (stacked-PoRep circuit: R1CS + GPU witness)
from . import sdr  # noqa: F401  (SDR labelling witness: SHA-256 labels of challenged nodes)
from .tuning import tune_clear, tune_get, tune_set, tuned  # noqa: F401  (test / A/B switches, csrc/tune.h)
