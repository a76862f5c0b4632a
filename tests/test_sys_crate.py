"""CPU: the Rust FFI crate at2v-sys against include/at2v.h. No cargo/rustc in this image, so
the check is textual: src/lib.rs's extern "C" block declares exactly the header's functions, with the same argument
counts and the same integer widths / pointer depths per argument and return value; the #[repr(C)] structs have the
header's fields in the header's order with the same widths; build.rs links libat2v the way the reference's build.rs
(/root/reference/build.rs:1-3) hosts its codegen step."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "at2v.h")
CRATE = os.path.join(ROOT, "at2v-sys")

C_BASE = {"int": "i32", "at2v_policy": "i32", "size_t": "usize", "uint8_t": "u8", "uint32_t": "u32",
          "uint64_t": "u64", "int32_t": "i32", "long": "long", "void": "void", "char": "char", "double": "f64",
          "at2v_ctx": "ctx", "at2v_opts": "opts", "at2v_info": "info", "at2v_queue": "queue",
          "at2v_queue_opts": "queue_opts", "at2v_queue_stats": "queue_stats", "at2v_ledger": "ledger",
          "at2v_send_asset_request": "send_asset_request", "at2v_full_transaction": "full_transaction",
          "at2v_apply_stats": "apply_stats"}
R_BASE = {"c_int": "i32", "i32": "i32", "usize": "usize", "u8": "u8", "u32": "u32", "u64": "u64", "c_long": "long",
          "c_void": "void", "c_char": "char", "f64": "f64", "At2vCtx": "ctx", "At2vOpts": "opts", "At2vInfo": "info",
          "At2vQueue": "queue", "At2vQueueOpts": "queue_opts", "At2vQueueStats": "queue_stats",
          "At2vLedger": "ledger", "At2vSendAssetRequest": "send_asset_request",
          "At2vFullTransaction": "full_transaction", "At2vApplyStats": "apply_stats"}


def c_type(decl: str) -> str:
    """'const uint8_t* pk' / 'uint8_t out[AT2V_UNIQUE_ID_BYTES]' / 'size_t n' -> canonical 'ptr u8' etc."""
    d = decl.replace("const", " ").strip()
    depth = d.count("*") + (1 if "[" in d else 0)
    d = re.sub(r"\[.*?\]", "", d).replace("*", " ")
    words = d.split()
    base = words[0] if len(words) == 1 or words[0] not in ("unsigned",) else words[1]
    return "ptr " * depth + C_BASE[base]


def r_type(t: str) -> str:
    t = t.strip()
    depth = 0
    while t.startswith("*"):
        depth += 1
        t = re.sub(r"^\*(const|mut)\s+", "", t)
    return "ptr " * depth + R_BASE[t]


def header_functions():
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    txt = re.sub(r"#.*", "", txt)
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(at2v_\w+)\s*\(([^;{]*?)\)\s*;", txt):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3).strip()
        ret = ret.split("\n")[-1].strip()
        argl = [] if args in ("", "void") else [c_type(a) for a in args.split(",")]
        out[name] = (c_type(ret + " x") if ret else "void", argl)
    return out


def crate_functions():
    src = open(os.path.join(CRATE, "src", "lib.rs")).read()
    block = src[src.index('extern "C" {'):]
    block = block[:block.index("\n}\n")]
    out = {}
    for m in re.finditer(r"pub fn (at2v_\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", block, flags=re.S):
        name, args, ret = m.group(1), m.group(2), m.group(3)
        argl = [r_type(a.split(":", 1)[1]) for a in args.split(",") if a.strip()]
        out[name] = (r_type(ret) if ret else "void", argl)
    return out


def test_extern_block_matches_header():
    h, r = header_functions(), crate_functions()
    import at2v
    assert sorted(h) == sorted(at2v.EXPORTED_SYMBOLS)
    assert sorted(r) == sorted(h), set(r) ^ set(h)
    for name in h:
        assert r[name] == h[name], (name, "rust", r[name], "header", h[name])


def header_structs():
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"typedef struct \{(.*?)\}\s*(at2v_\w+);", txt, flags=re.S):
        fields = []
        for line in m.group(1).split(";"):
            line = " ".join(line.replace("const ", " ").split())
            if not line:
                continue
            # "uint64_t submitted, completed" / "const uint8_t* sender" / "uint8_t sender[32]"
            mm = re.match(r"(\w+)\s*(\**)\s*(.*)", line)
            base, stars, rest = C_BASE[mm.group(1)], len(mm.group(2)), mm.group(3)
            for nm in rest.split(","):
                nm = nm.strip()
                arr = re.search(r"\[(\d+)\]", nm)
                star = stars + nm.count("*")
                nm = re.sub(r"\[.*?\]|\*", "", nm).strip()
                fields.append((nm, ("ptr " * star + base) + (f"[{arr.group(1)}]" if arr else "")))
        out[m.group(2)] = fields
    return out


def crate_structs():
    src = open(os.path.join(CRATE, "src", "lib.rs")).read()
    out = {}
    for m in re.finditer(r"pub struct (At2v\w+) \{(.*?)\}", src, flags=re.S):
        fields = []
        for f in re.finditer(r"pub (\w+):\s*([^,]+),", m.group(2)):
            t = f.group(2).strip()
            arr = re.match(r"\[(\w+);\s*(\d+)\]", t)
            fields.append((f.group(1), (r_type(arr.group(1)) + f"[{arr.group(2)}]") if arr else r_type(t)))
        if fields:
            out[m.group(1)] = fields
    return out


def test_repr_c_structs_match_header():
    h, r = header_structs(), crate_structs()
    pairs = {"at2v_opts": "At2vOpts", "at2v_info": "At2vInfo", "at2v_queue_opts": "At2vQueueOpts",
             "at2v_queue_stats": "At2vQueueStats", "at2v_send_asset_request": "At2vSendAssetRequest",
             "at2v_full_transaction": "At2vFullTransaction", "at2v_apply_stats": "At2vApplyStats"}
    assert set(h) == set(pairs), set(h) ^ set(pairs)
    for c, rs in pairs.items():
        assert r[rs] == h[c], (c, r[rs], h[c])


def test_constants_match_header():
    txt = open(HEADER).read()
    src = open(os.path.join(CRATE, "src", "lib.rs")).read()
    consts = dict(re.findall(r"\b(AT2V_[A-Z0-9_]+)\s*=\s*(-?\d+)", txt))
    consts.update(re.findall(r"#define (AT2V_[A-Z0-9_]+) ((?:0x)?[0-9a-fA-F]+)u?\b", txt))
    rust = dict(re.findall(r"pub const (AT2V_[A-Z0-9_]+): \w+ = (-?(?:0x)?[0-9a-f]+);", src))
    for k, v in consts.items():
        assert k in rust, k
        assert int(rust[k], 0) == int(v, 0), (k, rust[k], v)


def test_build_script_links_libat2v():
    b = open(os.path.join(CRATE, "build.rs")).read()
    assert "cargo:rustc-link-lib=dylib=at2v" in b and "cargo:rustc-link-search=native=" in b
    assert "AT2V_LIB_DIR" in b
    toml = open(os.path.join(CRATE, "Cargo.toml")).read()
    assert 'links = "at2v"' in toml and 'build = "build.rs"' in toml


def _rust_blocks_of_integration_md():
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    return re.findall(r"```rust\n(.*?)```", txt, flags=re.S)


def _struct_literals(src: str):
    """Every `At2vX { ... }` struct EXPRESSION in Rust source (definitions `struct At2vX {` excluded): yields
    (struct name, named fields, base expression or None). Handles `field: expr`, shorthand `field` and `..base`."""
    for m in re.finditer(r"(?<![\w])(At2v\w+)\s*\{", src):
        before = src[max(0, m.start() - 12):m.start()]
        if re.search(r"(struct|for|impl)\s+$", before):  # a definition or an `impl Trait for At2vX {` block
            continue
        i, depth = m.end(), 1
        while depth:
            depth += {"{": 1, "}": -1}.get(src[i], 0)
            i += 1
        body = src[m.end():i - 1]
        if not body.strip():  # `At2vFoo {}` would be a unit-like literal; none expected
            yield m.group(1), set(), None
            continue
        # split the top level on commas
        parts, cur, d = [], "", 0
        for ch in body:
            d += {"(": 1, "[": 1, "{": 1, ")": -1, "]": -1, "}": -1}.get(ch, 0)
            if ch == "," and d == 0:
                parts.append(cur)
                cur = ""
            else:
                cur += ch
        parts.append(cur)
        names, base = set(), None
        for p in (x.strip() for x in parts):
            if not p:
                continue
            if p.startswith(".."):
                base = p[2:].strip()
            else:
                names.add(p.split(":", 1)[0].strip())
        yield m.group(1), names, base


def _default_structs(src: str):
    """structs with a Default: derived, or a hand-written `impl Default for` (At2vOpts since ABI v6: num_gpus = 1)"""
    return (set(re.findall(r"#\[derive\([^)]*\bDefault\b[^)]*\)\]\s*pub struct (At2v\w+)", src))
            | set(re.findall(r"impl\s+Default\s+for\s+(At2v\w+)", src)))


def check_struct_literals(src: str, fields: dict, defaults: set):
    """every struct literal names exactly the struct's fields (or a subset plus `..Default::default()` on a struct
    that derives Default); returns the list of violations"""
    bad = []
    for name, names, base in _struct_literals(src):
        want = {f for f, _ in fields.get(name, [])}
        if name not in fields:
            bad.append((name, "unknown struct"))
        elif base is None and names != want:
            bad.append((name, "fields", sorted(names ^ want)))
        elif base is not None and (not names <= want or (base == "Default::default()" and name not in defaults)):
            bad.append((name, "base", sorted(names - want), base))
    return bad


def test_struct_literals_name_every_field():
    """`At2vOpts { device, num_gpus, policy }` (4-field struct) passed the declaration checks while rustc
    would reject it (E0063). Every struct literal in lib.rs and in INTEGRATION.md's Rust blocks must name exactly
    the fields the header gives the struct."""
    src = open(os.path.join(CRATE, "src", "lib.rs")).read()
    fields = crate_structs()
    assert fields["At2vOpts"] == [(f, t) for f, t in header_structs()["at2v_opts"]]
    defaults = _default_structs(src)
    assert check_struct_literals(src, fields, defaults) == []
    for block in _rust_blocks_of_integration_md():
        assert check_struct_literals(block, fields, defaults) == [], block


def test_struct_literal_check_catches_round2_defect():
    """the check above fails on round 2's BatchVerifier::new (the literal without small_batch_max)"""
    old = "let opts = At2vOpts { device, num_gpus, policy };"
    fields = crate_structs()
    assert check_struct_literals(old, fields, set())
    assert check_struct_literals("At2vOpts { device, num_gpus, policy, ..Default::default() }", fields,
                                 {"At2vOpts"}) == []
    assert check_struct_literals("At2vOpts { device, ..Default::default() }", fields, set())  # no Default derive


def test_integration_md_struct_definitions_match_header():
    """`pub struct At2v.. { .. }` re-declared in INTEGRATION.md's Rust blocks match the header too"""
    h = header_structs()
    pairs = {"At2vOpts": "at2v_opts", "At2vInfo": "at2v_info", "At2vQueueOpts": "at2v_queue_opts",
             "At2vQueueStats": "at2v_queue_stats"}
    for block in _rust_blocks_of_integration_md():
        for m in re.finditer(r"pub struct (At2v\w+)\s*\{(.*?)\}", block, flags=re.S):
            if m.group(1) not in pairs:
                continue
            got = [(f.group(1), r_type(f.group(2).strip())) for f in re.finditer(r"pub (\w+):\s*([^,}]+)", m.group(2))]
            assert got == h[pairs[m.group(1)]], (m.group(1), got)


def test_safe_layer_checks_abi_version():
    src = open(os.path.join(CRATE, "src", "lib.rs")).read()
    v = re.search(r"#define AT2V_ABI_VERSION (\d+)\b", open(HEADER).read()).group(1)
    assert f"pub const AT2V_ABI_VERSION: c_int = {v};" in src
    import at2v
    assert int(v) == at2v.ABI_VERSION
    for ctor in ("impl BatchVerifier", "impl Queue"):
        body = src[src.index(ctor):]
        body = body[:body.index("\n}\n")]
        assert "check_abi()?" in body, ctor


def test_safe_wrappers_check_offsets_against_msg():
    """the safe BatchVerifier::verify and Queue::submit hand msg.as_ptr() to C functions that read
    message bytes up to msg_off[n] with no length argument. Both must go through check_records, which refuses
    decreasing offsets and msg_off[n] > msg.len() (a #[test] in the crate covers it; no cargo here, so textually)."""
    src = open(os.path.join(CRATE, "src", "lib.rs")).read()
    fn = src[src.index("fn check_records("):]
    fn = fn[:fn.index("\n}\n")]
    assert "w[1] < w[0]" in fn and "msg.len()" in fn
    for wrapper in ("pub fn verify(", "pub fn submit("):
        body = src[src.index(wrapper):]
        body = body[:body.index("\n    }\n")]
        assert "check_records(pk, sig, msg, msg_off)?" in body, wrapper
    assert "fn safe_layer_rejects_offsets_outside_msg" in src and "&[0, 5]" in src
