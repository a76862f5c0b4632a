// build.rs — link libat2v.so (built by `make -C at2-node_amd`: hipcc for gfx950, RCCL from /opt/rocm/lib).
// AT2V_LIB_DIR overrides the location; the rpath lets the server binary find the library at run time.
// In the at2-node reference this is what its own build.rs (/root/reference/build.rs:1-3, tonic_build only)
// would gain if the binding lived in-tree instead of in this -sys crate.
use std::env;
use std::path::PathBuf;

fn main() {
    let dir = env::var("AT2V_LIB_DIR").map(PathBuf::from).unwrap_or_else(|_| {
        PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap()).join("../at2-node_amd/at2v")
    });
    let rocm = env::var("ROCM_PATH").unwrap_or_else(|_| "/opt/rocm".to_string());
    println!("cargo:rustc-link-search=native={}", dir.display());
    println!("cargo:rustc-link-lib=dylib=at2v");
    println!("cargo:rustc-link-search=native={}/lib", rocm);
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", dir.display());
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}/lib", rocm);
    println!("cargo:rerun-if-env-changed=AT2V_LIB_DIR");
    println!("cargo:rerun-if-env-changed=ROCM_PATH");
    println!("cargo:rerun-if-changed=../include/at2v.h");
}
