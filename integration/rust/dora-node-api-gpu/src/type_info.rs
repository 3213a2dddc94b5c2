//! The C ABI's serialized ArrowTypeInfo (`include/dora_gpu.h`, `dora_gpu_plan_type_info`) and
//! `dora_message::metadata::ArrowTypeInfo` (`libraries/message/src/metadata.rs:51-59`).
//!
//! Little-endian layout, per node:
//!   u32 n + n bytes   data_type as a schema tree: str format, str name, i64 flags,
//!                     u8 has_meta [str meta (Arrow C metadata blob)], u32 n_children x tree,
//!                     u8 has_dict [tree]                    (str = u32 n + n bytes)
//!   u64 len, u64 null_count
//!   u8 validity tag:  0 none | 1 u64 n + n bytes (inline, the reference's Option<Vec<u8>>)
//!                     | 2 u64 offset + u64 len (the bitmap lives in the sample's tail)
//!   u64 offset, u32 n_buffers x (u64 offset, u64 len), u32 n_children x node
//!
//! The data type travels as the Arrow C schema tree rather than bincode of `DataType`: the C
//! side has no serde.  Both directions go through `arrow_schema::ffi::FFI_ArrowSchema`, so the
//! mapping is arrow-rs's own C-interface mapping.
use std::collections::HashMap;

use arrow_schema::ffi::{FFI_ArrowSchema, Flags};
use arrow_schema::DataType;
use dora_message::metadata::{ArrowTypeInfo, BufferOffset};
use eyre::{bail, eyre, Context, Result};

struct Reader<'a> {
    b: &'a [u8],
    i: usize,
}

impl<'a> Reader<'a> {
    fn take(&mut self, n: usize) -> Result<&'a [u8]> {
        let end = self.i.checked_add(n).ok_or_else(|| eyre!("type info: length overflow"))?;
        let s = self.b.get(self.i..end).ok_or_else(|| eyre!("type info: truncated"))?;
        self.i = end;
        Ok(s)
    }
    fn u8(&mut self) -> Result<u8> {
        Ok(self.take(1)?[0])
    }
    fn u32(&mut self) -> Result<u32> {
        Ok(u32::from_le_bytes(self.take(4)?.try_into().unwrap()))
    }
    fn u64(&mut self) -> Result<u64> {
        Ok(u64::from_le_bytes(self.take(8)?.try_into().unwrap()))
    }
    fn i64(&mut self) -> Result<i64> {
        Ok(i64::from_le_bytes(self.take(8)?.try_into().unwrap()))
    }
    fn str(&mut self) -> Result<&'a [u8]> {
        let n = self.u32()? as usize;
        self.take(n)
    }
    fn usize(&mut self) -> Result<usize> {
        usize::try_from(self.u64()?).context("type info: value exceeds usize")
    }
}

/// Arrow C metadata blob (i32 n, then n x (i32 klen, key, i32 vlen, value)) as a map.
fn parse_c_metadata(m: &[u8]) -> Result<HashMap<String, String>> {
    let mut r = Reader { b: m, i: 0 };
    let rd_i32 = |r: &mut Reader| -> Result<usize> {
        let v = i32::from_le_bytes(r.take(4)?.try_into().unwrap());
        usize::try_from(v).context("negative length in schema metadata")
    };
    let n = rd_i32(&mut r)?;
    let mut out = HashMap::with_capacity(n);
    for _ in 0..n {
        let kl = rd_i32(&mut r)?;
        let k = String::from_utf8(r.take(kl)?.to_vec())?;
        let vl = rd_i32(&mut r)?;
        let v = String::from_utf8(r.take(vl)?.to_vec())?;
        out.insert(k, v);
    }
    Ok(out)
}

fn c_metadata(m: &HashMap<String, String>) -> Vec<u8> {
    let mut o = (m.len() as i32).to_le_bytes().to_vec();
    let mut keys: Vec<_> = m.keys().collect();
    keys.sort();
    for k in keys {
        let v = &m[k];
        o.extend_from_slice(&(k.len() as i32).to_le_bytes());
        o.extend_from_slice(k.as_bytes());
        o.extend_from_slice(&(v.len() as i32).to_le_bytes());
        o.extend_from_slice(v.as_bytes());
    }
    o
}

fn schema_tree(r: &mut Reader, top: bool) -> Result<FFI_ArrowSchema> {
    let format = std::str::from_utf8(r.str()?)?.to_owned();
    let name = std::str::from_utf8(r.str()?)?.to_owned();
    let flags = r.i64()?;
    let meta = if r.u8()? != 0 { Some(parse_c_metadata(r.str()?)?) } else { None };
    let n_children = r.u32()?;
    let mut children = Vec::with_capacity(n_children as usize);
    for _ in 0..n_children {
        children.push(schema_tree(r, false)?);
    }
    let dictionary = if r.u8()? != 0 { Some(schema_tree(r, false)?) } else { None };
    let mut s = FFI_ArrowSchema::try_new(&format, children, dictionary)?;
    if !top {
        s = s.with_name(&name)?;
    }
    s = s.with_flags(Flags::from_bits(flags).ok_or_else(|| eyre!("schema flags {flags:#x}"))?)?;
    if let Some(m) = meta {
        s = s.with_metadata(m)?;
    }
    Ok(s)
}

fn put_str(o: &mut Vec<u8>, s: &[u8]) {
    o.extend_from_slice(&(s.len() as u32).to_le_bytes());
    o.extend_from_slice(s);
}

fn put_schema_tree(s: &FFI_ArrowSchema, top: bool, o: &mut Vec<u8>) -> Result<()> {
    put_str(o, s.format().as_bytes());
    put_str(o, if top { b"" } else { s.name().unwrap_or("").as_bytes() });
    let mut flags = s.flags().map(|f| f.bits()).unwrap_or(0);
    if top {
        // the top level carries only the type-relevant flags (dictionary ordered, keys sorted)
        flags &= (Flags::DICTIONARY_ORDERED | Flags::MAP_KEYS_SORTED).bits();
    }
    o.extend_from_slice(&flags.to_le_bytes());
    let meta = if top { HashMap::new() } else { s.metadata()? };
    o.push(u8::from(!meta.is_empty()));
    if !meta.is_empty() {
        put_str(o, &c_metadata(&meta));
    }
    o.extend_from_slice(&(s.n_children() as u32).to_le_bytes());
    for i in 0..s.n_children() {
        put_schema_tree(s.child(i), false, o)?;
    }
    o.push(u8::from(s.dictionary().is_some()));
    if let Some(d) = s.dictionary() {
        put_schema_tree(d, false, o)?;
    }
    Ok(())
}

/// Where a validity bitmap of tag 2 is read from: `(offset, len)` in the received sample.  For
/// a device sample this is one device-to-host copy (`dora_gpu_memcpy_async` + sync).
pub type TailReader<'a> = dyn FnMut(usize, usize) -> Result<Vec<u8>> + 'a;

fn node(r: &mut Reader, tail: &mut TailReader) -> Result<ArrowTypeInfo> {
    let mut sr = Reader { b: r.str()?, i: 0 };
    let data_type = DataType::try_from(&schema_tree(&mut sr, true)?)?;
    let len = r.usize()?;
    let null_count = r.usize()?;
    let validity = match r.u8()? {
        0 => None,
        1 => {
            let n = r.usize()?;
            Some(r.take(n)?.to_vec())
        }
        2 => {
            let (off, n) = (r.usize()?, r.usize()?);
            Some(tail(off, n)?)
        }
        t => bail!("type info: validity tag {t}"),
    };
    let offset = r.usize()?;
    let nb = r.u32()?;
    let mut buffer_offsets = Vec::with_capacity(nb as usize);
    for _ in 0..nb {
        buffer_offsets.push(BufferOffset { offset: r.usize()?, len: r.usize()? });
    }
    let nc = r.u32()?;
    let mut child_data = Vec::with_capacity(nc as usize);
    for _ in 0..nc {
        child_data.push(node(r, tail)?);
    }
    Ok(ArrowTypeInfo { data_type, len, null_count, validity, offset, buffer_offsets, child_data })
}

/// Decode the C ABI's type info bytes (`dora_gpu_plan_type_info`, `dora_event_type_info`,
/// descriptors on the wire) into the reference `ArrowTypeInfo`.  Bitmaps that travelled in the
/// sample's tail (tag 2) are fetched through `tail`; `dora_event_type_info` already returns
/// the inline form, for which `tail` is never called.
pub fn decode(bytes: &[u8], tail: &mut TailReader) -> Result<ArrowTypeInfo> {
    let mut r = Reader { b: bytes, i: 0 };
    let t = node(&mut r, tail)?;
    if r.i != bytes.len() {
        bail!("type info: {} trailing bytes", bytes.len() - r.i);
    }
    Ok(t)
}

/// Decode a type info whose bitmaps are all inline (tag 2 is an error).
pub fn decode_inline(bytes: &[u8]) -> Result<ArrowTypeInfo> {
    decode(bytes, &mut |_, _| bail!("validity in the sample tail: use decode with a tail reader"))
}

/// Encode the reference `ArrowTypeInfo` into the C ABI form (validity inline, tag 1), e.g. for
/// `dora_node_send_output_sample` of a sample a Rust node filled itself.
pub fn encode(t: &ArrowTypeInfo) -> Result<Vec<u8>> {
    let mut o = Vec::new();
    encode_into(t, &mut o)?;
    Ok(o)
}

fn encode_into(t: &ArrowTypeInfo, o: &mut Vec<u8>) -> Result<()> {
    let mut tree = Vec::new();
    put_schema_tree(&FFI_ArrowSchema::try_from(&t.data_type)?, true, &mut tree)?;
    put_str(o, &tree);
    o.extend_from_slice(&(t.len as u64).to_le_bytes());
    o.extend_from_slice(&(t.null_count as u64).to_le_bytes());
    match &t.validity {
        None => o.push(0),
        Some(v) => {
            o.push(1);
            o.extend_from_slice(&(v.len() as u64).to_le_bytes());
            o.extend_from_slice(v);
        }
    }
    o.extend_from_slice(&(t.offset as u64).to_le_bytes());
    o.extend_from_slice(&(t.buffer_offsets.len() as u32).to_le_bytes());
    for b in &t.buffer_offsets {
        o.extend_from_slice(&(b.offset as u64).to_le_bytes());
        o.extend_from_slice(&(b.len as u64).to_le_bytes());
    }
    o.extend_from_slice(&(t.child_data.len() as u32).to_le_bytes());
    for c in &t.child_data {
        encode_into(c, o)?;
    }
    Ok(())
}

#[cfg(test)]
mod tests {
    use super::*;

    #[test]
    fn byte_array_roundtrip() {
        let t = ArrowTypeInfo::byte_array(4096);
        let b = encode(&t).unwrap();
        assert_eq!(decode_inline(&b).unwrap(), t);
    }

    #[test]
    fn tag2_reads_the_tail() {
        let mut t = ArrowTypeInfo::byte_array(9);
        t.null_count = 1;
        t.validity = Some(vec![0xfe, 0x01]);
        let mut b = encode(&t).unwrap();
        // rewrite tag 1 (inline, 2 bytes) as tag 2 (offset 64, len 2)
        let at = b.len() - (1 + 8 + 2) - 8 - 4 - 16 - 4;
        b.splice(at..at + 11, [vec![2u8], 64u64.to_le_bytes().to_vec(), 2u64.to_le_bytes().to_vec()].concat());
        let got = decode(&b, &mut |off, n| {
            assert_eq!((off, n), (64, 2));
            Ok(vec![0xfe, 0x01])
        })
        .unwrap();
        assert_eq!(got, t);
    }
}
