// Link libhec.so (built by `make` at the repo root into helyim_amd/).
// HEC_LIB_DIR overrides the search path.
fn main() {
    let dir = std::env::var("HEC_LIB_DIR").unwrap_or_else(|_| {
        let root = std::path::Path::new(env!("CARGO_MANIFEST_DIR")).join("../../helyim_amd");
        root.to_string_lossy().into_owned()
    });
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=hec");
    println!("cargo:rerun-if-env-changed=HEC_LIB_DIR");
}
