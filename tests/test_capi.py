"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports
every symbol declared in include/gasalx.h, the reference-compatible C++ API
symbols are present, and host-side logic (batch layout, CIGAR decoding,
synthetic workloads) behaves like the reference.  No compute calls."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import gasal_ffi as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_c_functions():
    src = open(os.path.join(ROOT, "include", "gasalx.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(gasalx_\w+)\s*\(", src, re.M)))


def test_lib_loads_and_exports_every_declared_symbol():
    lib = G.lib()
    declared = _declared_c_functions()
    assert len(declared) >= 12
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(G.EXPORTS)


def test_cpp_api_symbols_present():
    out = subprocess.run(["nm", "-DC", G.LIB_PATH], capture_output=True, text=True, check=True).stdout
    for sym in ("gasal_init_gpu_storage_v(int)", "gasal_init_streams(", "gasal_destroy_streams(",
                "gasal_destroy_gpu_storage_v(", "gasal_host_batch_fill(", "gasal_host_batch_add(",
                "gasal_host_batch_addbase(", "gasal_host_batch_new(", "gasal_host_batch_destroy(",
                "gasal_host_batch_reset(", "gasal_host_batch_getlast(", "gasal_host_batch_print(",
                "gasal_host_batch_printall(", "gasal_host_alns_resize(", "gasal_op_fill(", "gasal_set_device(",
                "gasal_copy_subst_scores(", "gasal_aln_async(", "gasal_is_aln_async_done(",
                "gasal_res_new_host(", "gasal_res_new_device(", "gasal_res_new_device_cpy(",
                "gasal_res_destroy_host(", "gasal_res_destroy_device(", "Parameters::Parameters(int, char**)",
                "Parameters::parse()", "gasal_gpu_mem_alloc(", "gasal_gpu_mem_free("):
        assert sym in out, sym


def test_abi_version():
    assert G.lib().gasalx_abi_version() == 1


def test_batch_layout_matches_host_batch_fill():
    # host_batch.cpp:100-102,137-150: pad with N_CODE to a multiple of 8
    b = G.Batch.from_pairs(["ACGTA", "ACGTACGT", "A"], ["GG", "T" * 9, "C" * 16])
    assert list(b.q_offsets) == [0, 8, 16] and list(b.q_lens) == [5, 8, 1]
    assert bytes(b.q_data[:8]) == b"ACGTANNN"
    assert list(b.t_offsets) == [0, 8, 24] and b.t_bytes == 40


def test_decode_cigar_merges_split_runs():
    # reversed bytes: count<<2|op; 63-runs of one op are merged when printed
    rev = np.array([(1 << 2) | 0, (63 << 2) | 0, (2 << 2) | 3, (5 << 2) | 0], np.uint8)
    assert G.decode_cigar(rev, 0, 4) == "5M2I64M"


def test_plan_selection_cpu_only():
    assert G.describe_plan(G.make_params(algo=G.LOCAL), 150, 150) == "wavefront16_local_G8R19"
    assert G.describe_plan(G.make_params(algo=G.LOCAL, match=2), 150, 150) == "wavefront16_local_u16_G8R19"
    # past the u16 range: f16 keys by 64-step segments (WF16_LOCAL_SEG); GASALX_KSEG=0: the int32 kernel
    assert G.describe_plan(G.make_params(algo=G.LOCAL, match=3), 150, 150) == "wavefront16_local_seg64_G8R19"
    assert G.describe_plan(G.make_params(algo=G.LOCAL), 300, 300) == "wavefront16_local_seg64_G16R20"
    assert G.describe_plan(G.make_params(algo=G.LOCAL, start_pos=G.WITH_TB), 150, 150) == "wavefront16_local_tb_dr_G8R20"
    assert G.describe_plan(G.make_params(algo=G.LOCAL, start_pos=G.WITH_TB, match=2), 150, 150) == \
        "wavefront_local_tb_keys_G8R20"
    assert G.describe_plan(G.make_params(algo=G.LOCAL, start_pos=G.WITH_START), 150, 150) == \
        "wavefront16_local_start_G8R19"
    assert G.describe_plan(G.make_params(algo=G.SEMI_GLOBAL, start_pos=G.WITH_START), 150, 182) == \
        "wavefront16_semi_start_G8R23"
    assert G.describe_plan(G.make_params(algo=G.SEMI_GLOBAL, start_pos=G.WITH_START, tail=G.QUERY), 150, 182) == \
        "generic_semi"
    assert G.describe_plan(G.make_params(algo=G.LOCAL, second_best=1), 150, 150) == "local16_second"
    assert G.describe_plan(G.make_params(algo=G.LOCAL, second_best=1, start_pos=G.WITH_START), 150, 150) == \
        "generic_local"
    assert G.describe_plan(G.make_params(algo=G.KSW), 150, 150) == "generic_ksw"
    assert G.describe_plan(G.make_params(algo=G.GLOBAL, start_pos=G.WITH_TB), 300, 300) == \
        "wavefront16_global_tbband_G16R20"
    assert G.describe_plan(G.make_params(algo=G.UNKNOWN), 10, 10) == "none"


def test_synthetic_workloads_deterministic():
    a = G.Batch.synth(2, 64, 0x5EED0002)
    b = G.Batch.synth(2, 64, 0x5EED0002)
    assert np.array_equal(a.q_data, b.q_data) and np.array_equal(a.t_data, b.t_data)
    assert set(a.q_lens) == {150} and set(a.t_lens) == {150} and a.q_bytes == 64 * 152
    c = G.Batch.synth(4, 32, 0x5EED0004)
    assert set(c.q_lens) == {150} and set(c.t_lens) == {182}


def test_pairhmm_params_match_oracle():
    import oracle as O
    bq = np.arange(0, 60, dtype=np.uint8)
    iq = np.full(60, 45, np.uint8)
    dq = np.full(60, 45, np.uint8)
    a = G.pairhmm_params(bq, iq, dq)
    b = O.pairhmm_params(bq, iq, dq)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_no_gpu_call_fails_loudly_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        G.Engine(0)


def test_synth_range_is_a_shard_of_the_global_batch():
    # pairs [start, start + n) generated alone equal the same pairs of the whole batch,
    # across a 65,536-pair block boundary (gasalx_synth_range: one generator per block)
    full = G.Batch.synth(1, 70000, 0x5EED0001)
    for start, n in ((0, 5), (65530, 12), (69990, 10)):
        part = G.Batch.synth(1, n, 0x5EED0001, start=start)
        sl = full.slice(start, start + n)
        assert np.array_equal(part.q_data, sl.q_data) and np.array_equal(part.t_data, sl.t_data)
        assert np.array_equal(part.q_offsets, sl.q_offsets) and np.array_equal(part.t_lens, sl.t_lens)
    assert G.synth_spec(4) == (150, 182) and G.synth_spec(1) == (64, 64)


def test_batch_slice_matches_subset():
    b = G.Batch.from_pairs(["ACGTA", "A" * 17, "CG", "T" * 8], ["GG", "C" * 9, "ACGTACGTA", "A"])
    for s, e in ((0, 4), (1, 3), (2, 2), (3, 4)):
        x, y = b.slice(s, e), b.subset(np.arange(s, e))
        assert x.n == y.n
        if x.n:
            assert np.array_equal(x.q_data, y.q_data) and np.array_equal(x.t_offsets, y.t_offsets)
            assert np.array_equal(x.q_lens, y.q_lens)


def test_pinned_host_lifetime_follows_its_arrays():
    # gasalx_host_alloc is exported; without a device it fails loudly, with one the
    # memory lives as long as any view (tests/test_gpu_parity.py covers the GPU side)
    import gc
    import weakref
    try:
        h = G.PinnedHost(64)
    except RuntimeError:
        pytest.skip("no HIP device for page-locked memory")
    view = h.array[8:16]
    ref = weakref.ref(h)
    h.close()
    del h
    gc.collect()
    assert ref() is not None          # the view still holds the owner
    view[:] = 7
    del view
    gc.collect()
    assert ref() is None


def test_reference_error_helpers_compile(tmp_path):
    # a caller written against the reference's gasal.h error helpers (gasal.h:15-34)
    # compiles unchanged against include/gasal_header.h
    src = tmp_path / "caller.cpp"
    src.write_text('#include "gasal_header.h"\n'
                   "int f() { hipError_t err; CHECKCUDAERROR(hipGetLastError());\n"
                   "          return CudaCheckKernelLaunch(); }\n")
    subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-c", str(src), "-o",
                    str(tmp_path / "caller.o")], check=True, capture_output=True)
