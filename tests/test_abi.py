"""The C-ABI library: builds for gfx950 (hipcc cross-compiles here), loads, and exports every symbol
include/ptls_mi355x.h declares; the header's picotls type mirror is layout-identical to the
reference's include/picotls.h.  No compute calls: these run without a GPU."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ptls_mi355x.h")
REF_INC = "/root/reference/include"


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    funcs = set(re.findall(r"\b(ptls_mi355x_\w+)\s*\(", src))
    objs = set()
    for m in re.finditer(r"extern\s+ptls_\w+_t\s+([^;]+);", src):
        objs |= {x.strip() for x in m.group(1).split(",")}
    return funcs, objs


def test_library_exports_every_declared_symbol(engine_lib):
    import rapido_amd
    funcs, objs = declared()
    assert funcs == set(rapido_amd.EXPORTED_FUNCTIONS)
    assert objs == set(rapido_amd.EXPORTED_OBJECTS)
    for name in funcs | objs:
        assert hasattr(engine_lib, name), name


def test_library_build_id_is_the_source_hash(engine_lib):
    """Build provenance: the library in the tree was built from the tree's sources (rapido_amd/build.py stamps it
    with their hash and rebuilds whenever the hash changes)."""
    import rapido_amd as ra
    from rapido_amd import build
    bid = ra.build_id()
    assert re.fullmatch(r"[0-9a-f]{16}", bid)
    assert bid == ra.source_build_id() == build.stamped_build_id()


def test_library_has_gfx950_code_object(engine_lib):
    """The fat binary embedded in the library carries a gfx950 code object (and only that target)."""
    import rapido_amd
    blob = open(rapido_amd.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"amdgcn-amd-amdhsa--gfx942" not in blob and b"amdgcn-amd-amdhsa--gfx90a" not in blob


def test_algorithm_objects_match_slot_contract(engine_lib):
    import rapido_amd as ra
    for name, ks in (("aes128gcm", 16), ("aes256gcm", 32)):
        a = ra.algorithm(name)
        assert a.key_size == ks and a.iv_size == 12 and a.tag_size == 16
        assert a.confidentiality_limit == 1 << 25 and a.integrity_limit == 1 << 54  # include/picotls.h:80-81
        assert a.name.decode() == ("AES128-GCM" if ks == 16 else "AES256-GCM")
        assert a.context_size >= C.sizeof(ra.AeadContext)
        assert a.ctr_cipher.contents.key_size == ks and a.ctr_cipher.contents.iv_size == 16
        # fusion leaves ecb_cipher NULL (lib/fusion.c:990, 1000); the generic suite (t/picotls.c:266-307) needs it,
        # with the shape of ptls_openssl_aes{128,256}ecb (lib/openssl.c:1580-1597)
        e = a.ecb_cipher.contents
        assert e.key_size == ks and e.block_size == 16 and e.iv_size == 0
        assert e.name.decode() == ("AES128-ECB" if ks == 16 else "AES256-ECB")
        assert e.context_size >= C.sizeof(ra.CipherContext)


def _compile_and_run(tmp_path, name, src, incs):
    c = tmp_path / (name + ".c")
    c.write_text(src)
    exe = tmp_path / name
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", *[f"-I{i}" for i in incs], str(c), "-o", str(exe)],
                   check=True)
    return subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout


LAYOUT_PROBE = r"""
#include <stdio.h>
#include <stddef.h>
%s
#define F(T, f) printf(#T "." #f " %%zu %%zu\n", offsetof(T, f), sizeof(((T *)0)->f));
int main(void) {
  printf("aead_ctx %%zu aead_algo %%zu cipher_ctx %%zu cipher_algo %%zu supp %%zu\n", sizeof(ptls_aead_context_t),
         sizeof(struct st_ptls_aead_algorithm_t), sizeof(ptls_cipher_context_t), sizeof(struct st_ptls_cipher_algorithm_t),
         sizeof(ptls_aead_supplementary_encryption_t));
  F(ptls_aead_context_t, algo) F(ptls_aead_context_t, dispose_crypto) F(ptls_aead_context_t, do_xor_iv)
  F(ptls_aead_context_t, do_encrypt_init) F(ptls_aead_context_t, do_encrypt_update) F(ptls_aead_context_t, do_encrypt_final)
  F(ptls_aead_context_t, do_encrypt) F(ptls_aead_context_t, do_decrypt)
  F(struct st_ptls_aead_algorithm_t, name) F(struct st_ptls_aead_algorithm_t, confidentiality_limit)
  F(struct st_ptls_aead_algorithm_t, integrity_limit) F(struct st_ptls_aead_algorithm_t, ctr_cipher)
  F(struct st_ptls_aead_algorithm_t, ecb_cipher) F(struct st_ptls_aead_algorithm_t, key_size)
  F(struct st_ptls_aead_algorithm_t, iv_size) F(struct st_ptls_aead_algorithm_t, tag_size)
  F(struct st_ptls_aead_algorithm_t, context_size) F(struct st_ptls_aead_algorithm_t, setup_crypto)
  F(ptls_cipher_context_t, algo) F(ptls_cipher_context_t, do_dispose) F(ptls_cipher_context_t, do_init)
  F(ptls_cipher_context_t, do_transform)
  F(struct st_ptls_cipher_algorithm_t, name) F(struct st_ptls_cipher_algorithm_t, key_size)
  F(struct st_ptls_cipher_algorithm_t, block_size) F(struct st_ptls_cipher_algorithm_t, iv_size)
  F(struct st_ptls_cipher_algorithm_t, context_size) F(struct st_ptls_cipher_algorithm_t, setup_crypto)
  F(ptls_aead_supplementary_encryption_t, ctx) F(ptls_aead_supplementary_encryption_t, input)
  F(ptls_aead_supplementary_encryption_t, output)
  return 0;
}
"""


def test_header_compiles_standalone_c_and_cxx(tmp_path):
    (tmp_path / "a.c").write_text('#include "ptls_mi355x.h"\nint main(void){return ptls_mi355x_aes128gcm.tag_size != 16;}\n')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", f"-I{ROOT}/include", str(tmp_path / "a.c")],
                   check=True)
    (tmp_path / "b.cpp").write_text('#include "ptls_mi355x.h"\nint main(){return (int)sizeof(ptls_mi355x_record_t) - 40;}\n')
    subprocess.run(["g++", "-std=c++11", "-Wall", "-Werror", "-fsyntax-only", f"-I{ROOT}/include", str(tmp_path / "b.cpp")],
                   check=True)


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_INC, "picotls.h")), reason="reference headers not present")
def test_mirror_layout_equals_reference_picotls_h(tmp_path):
    ours = _compile_and_run(tmp_path, "ours", LAYOUT_PROBE % '#include "ptls_mi355x.h"', [f"{ROOT}/include"])
    ref = _compile_and_run(tmp_path, "ref", LAYOUT_PROBE % '#include "picotls.h"', [REF_INC])
    assert ours == ref
    # and the header is usable after the real picotls.h (its mirror then steps aside)
    both = _compile_and_run(tmp_path, "both", LAYOUT_PROBE % '#include "picotls.h"\n#include "ptls_mi355x.h"',
                            [REF_INC, f"{ROOT}/include"])
    assert both == ref


def test_ctypes_mirror_sizes(tmp_path):
    import rapido_amd as ra
    out = _compile_and_run(tmp_path, "sz", LAYOUT_PROBE % '#include "ptls_mi355x.h"', [f"{ROOT}/include"])
    first = out.splitlines()[0].split()
    sizes = dict(zip(first[0::2], map(int, first[1::2])))
    assert sizes["aead_ctx"] == C.sizeof(ra.AeadContext)
    assert sizes["aead_algo"] == C.sizeof(ra.AeadAlgorithm)
    assert sizes["cipher_ctx"] == C.sizeof(ra.CipherContext)
    assert sizes["cipher_algo"] == C.sizeof(ra.CipherAlgorithm)
    assert sizes["supp"] == C.sizeof(ra.SupplementaryEncryption)


def test_no_oracle_in_product():
    """The product library and package never reference the oracle (checker only)."""
    import rapido_amd
    blob = open(rapido_amd.LIB_PATH, "rb").read()
    assert b"oracle_gcm" not in blob and b"ref_seal" not in blob
    for dirpath, _, files in os.walk(os.path.join(ROOT, "rapido_amd")):
        for f in files:
            if f.endswith((".py", ".c", ".h", ".hip", ".cpp")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in txt and "from oracle" not in txt, f
