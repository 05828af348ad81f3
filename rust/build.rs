// build.rs -- links the reference crate against libvsg.so (the MI355X-native
// replacement of the `usearch` crate, include/vsg.h).  Drop this file next to
// /root/reference/Cargo.toml (or merge it into an existing build.rs).
//
// libvsg.so is built by `make -C vector-store-text_amd -j16` (hipcc, gfx950).
// VSG_LIB_DIR overrides the directory that holds it.
fn main() {
    let dir = std::env::var("VSG_LIB_DIR").unwrap_or_else(|_| "vector-store-text_amd/lib".to_string());
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=vsg");
    // the HIP runtime libvsg.so depends on
    println!("cargo:rustc-link-search=native=/opt/rocm/lib");
    println!("cargo:rustc-link-lib=dylib=amdhip64");
    println!("cargo:rerun-if-changed=include/vsg.h");
    println!("cargo:rerun-if-env-changed=VSG_LIB_DIR");
}
