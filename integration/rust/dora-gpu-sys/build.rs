//! Builds libdora_gpu as a static library with hipcc (gfx950), no CMake, no CUDA shims — the
//! same recipe as dora_amd/build.py — or links a prebuilt one.
//!
//!   DORA_GPU_LIB_DIR=<dir with libdora_gpu.so>   link the prebuilt shared library (rpath set)
//!   DORA_GPU_SRC=<repo root>                      where dora_amd/csrc and include/ live
//!                                                 (default: three levels above this crate)
//!   HIPCC=<path>                                  default /opt/rocm/bin/hipcc
use std::env;
use std::fs;
use std::path::{Path, PathBuf};
use std::process::Command;

const ARCH: &str = "gfx950";
const LIB_SOURCES: &[&str] = &[
    "runtime.cpp", "plan.cpp", "device_array.cpp", "kernels.hip", "shm.cpp", "bcast.cpp",
    "operator_api.cpp", "stdout_capture.cpp", "wire.cpp", "trace.cpp", "daemon.cpp", "node.cpp",
    "aql.cpp", "interdaemon.cpp",
];

fn run(cmd: &mut Command) {
    let status = cmd.status().unwrap_or_else(|e| panic!("failed to start {:?}: {e}", cmd));
    assert!(status.success(), "{:?} failed with {status}", cmd);
}

fn main() {
    println!("cargo:rerun-if-env-changed=DORA_GPU_LIB_DIR");
    println!("cargo:rerun-if-env-changed=DORA_GPU_SRC");
    println!("cargo:rerun-if-env-changed=HIPCC");
    let rocm_lib = "/opt/rocm/lib";

    if let Ok(dir) = env::var("DORA_GPU_LIB_DIR") {
        println!("cargo:rustc-link-search=native={dir}");
        println!("cargo:rustc-link-lib=dylib=dora_gpu");
        println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
        return;
    }

    let manifest = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap());
    let src_root = env::var("DORA_GPU_SRC")
        .map(PathBuf::from)
        .unwrap_or_else(|_| manifest.join("../../.."));
    let csrc = src_root.join("dora_amd/csrc");
    let include = src_root.join("include");
    let hipcc = env::var("HIPCC").unwrap_or_else(|_| "/opt/rocm/bin/hipcc".into());
    let out = PathBuf::from(env::var("OUT_DIR").unwrap());
    println!("cargo:rerun-if-changed={}", csrc.display());
    println!("cargo:rerun-if-changed={}", include.display());

    let common = |c: &mut Command| {
        c.args(["-O3", "-std=c++17", "-fPIC"])
            .arg(format!("-I{}", include.display()))
            .arg(format!("-I{}", csrc.display()));
    };
    let mut objs: Vec<PathBuf> = Vec::new();
    for s in LIB_SOURCES {
        let src = csrc.join(s);
        let obj = out.join(format!("{s}.o"));
        let mut c = Command::new(&hipcc);
        if s.ends_with(".hip") {
            c.args(["-x", "hip"]).arg(format!("--offload-arch={ARCH}"));
        } else {
            c.args(["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]);
        }
        common(&mut c);
        c.arg("-c").arg(&src).arg("-o").arg(&obj);
        run(&mut c);
        objs.push(obj);
    }

    // The AQL pack kernels: a raw gfx950 code object (kernel-argument preload for the
    // single-segment kernels), embedded with .incbin as dora_aql_code_object[_end].
    let co = out.join("aql_kernels.co");
    let mut c = Command::new(&hipcc);
    c.args(["--genco", "--offload-device-only", "--no-gpu-bundle-output", "-O3", "-std=c++17"])
        .arg(format!("--offload-arch={ARCH}"))
        .args(["-mllvm", "-amdgpu-kernarg-preload-count=14"])
        .arg(format!("-I{}", include.display()))
        .arg(format!("-I{}", csrc.display()))
        .arg(csrc.join("aql_kernels.hip"))
        .arg("-o")
        .arg(&co);
    run(&mut c);
    let asm = out.join("aql_blob.S");
    fs::write(
        &asm,
        format!(
            ".section .rodata\n.p2align 12\n.globl dora_aql_code_object\ndora_aql_code_object:\n\
             .incbin \"{}\"\n.globl dora_aql_code_object_end\ndora_aql_code_object_end:\n\
             .section .note.GNU-stack,\"\",@progbits\n",
            co.display()
        ),
    )
    .unwrap();
    let blob = out.join("aql_blob.o");
    run(Command::new(&hipcc).args(["-c", "-x", "assembler-with-cpp"]).arg(&asm).arg("-o").arg(&blob));
    objs.push(blob);

    let lib = out.join("libdora_gpu.a");
    let _ = fs::remove_file(&lib);
    run(Command::new("ar").arg("crs").arg(&lib).args(objs.iter().map(|p| p.as_path())));
    link(&out, rocm_lib);
}

fn link(out: &Path, rocm_lib: &str) {
    println!("cargo:rustc-link-search=native={}", out.display());
    println!("cargo:rustc-link-lib=static=dora_gpu");
    println!("cargo:rustc-link-search=native={rocm_lib}");
    // the HIP runtime (device code registration of kernels.hip), ROCr for the AQL queues
    for l in ["amdhip64", "hsa-runtime64", "stdc++", "dl", "pthread", "rt"] {
        println!("cargo:rustc-link-lib=dylib={l}");
    }
    println!("cargo:rustc-link-arg=-Wl,-rpath,{rocm_lib}");
}
