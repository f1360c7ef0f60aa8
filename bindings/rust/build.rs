// Links the prebuilt HIP library (rusty_enet_amd/lib/libenet_crc_amd.so, built by
// `make` at the repo root).  Override the directory with ENET_CRC_AMD_LIB_DIR.
fn main() {
    let dir = std::env::var("ENET_CRC_AMD_LIB_DIR").unwrap_or_else(|_| {
        let manifest = std::env::var("CARGO_MANIFEST_DIR").unwrap();
        format!("{manifest}/../../rusty_enet_amd/lib")
    });
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=enet_crc_amd");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    println!("cargo:rerun-if-env-changed=ENET_CRC_AMD_LIB_DIR");
}
