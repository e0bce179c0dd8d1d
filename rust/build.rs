// build.rs for syncr with the `gpu` feature (integration/file_operations.diff
// adds `build = "build.rs"` to Cargo.toml): links libsyncr_cdc.so, the MI355X
// chunker built by `python -m syncr_amd.build` (hipcc --offload-arch=gfx950).
//
//   SYNCR_CDC_LIB_DIR   directory holding libsyncr_cdc.so (default: the
//                       repository's syncr_amd/ next to this crate)
//   ROCM_PATH           ROCm install (default /opt/rocm): libamdhip64
//
// Without the feature nothing is linked and syncr builds exactly as before.
use std::env;
use std::path::PathBuf;

fn main() {
    println!("cargo:rerun-if-changed=build.rs");
    println!("cargo:rerun-if-env-changed=SYNCR_CDC_LIB_DIR");
    println!("cargo:rerun-if-env-changed=ROCM_PATH");
    if env::var_os("CARGO_FEATURE_GPU").is_none() {
        return;
    }
    let lib_dir = env::var_os("SYNCR_CDC_LIB_DIR").map(PathBuf::from).unwrap_or_else(|| {
        PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap()).join("..").join("syncr_amd")
    });
    let lib = lib_dir.join("libsyncr_cdc.so");
    if !lib.exists() {
        panic!("feature `gpu`: {} not found; build it with `python -m syncr_amd.build` and set \
                SYNCR_CDC_LIB_DIR", lib.display());
    }
    let rocm = env::var_os("ROCM_PATH").map(PathBuf::from).unwrap_or_else(|| PathBuf::from("/opt/rocm"));
    println!("cargo:rustc-link-search=native={}", lib_dir.display());
    println!("cargo:rustc-link-search=native={}", rocm.join("lib").display());
    println!("cargo:rustc-link-lib=dylib=syncr_cdc");
    println!("cargo:rustc-link-lib=dylib=amdhip64");
    // the binary finds the library where it was linked from
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", lib_dir.display());
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", rocm.join("lib").display());
}
