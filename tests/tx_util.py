"""Helpers shared by the tx-layer tests: fixture headers -> TX_HEADER records."""
import numpy as np

TX_HEADER = np.dtype([("id", "<u8"), ("ts", "<i8"), ("bl_tx_id", "<u8"), ("bl_root", "u1", 32),
                      ("prev_alh", "u1", 32), ("eh", "u1", 32), ("version", "<u4"),
                      ("nentries", "<u4"), ("md_len", "<u4"), ("md_off", "<u4")])


def headers_from_fixture(txs):
    """-> (records[n] of TX_HEADER, md_blob bytes, stored alh[n] as bytes)"""
    recs = np.zeros(len(txs), TX_HEADER)
    blob = bytearray()
    alhs = []
    for k, t in enumerate(txs):
        h = t["header"]
        r = recs[k]
        r["id"], r["ts"], r["bl_tx_id"] = h["id"], h["ts"], h["bltxid"]
        r["bl_root"] = np.frombuffer(bytes.fromhex(h["blroot"]), np.uint8)
        r["prev_alh"] = np.frombuffer(bytes.fromhex(h["prevalh"]), np.uint8)
        r["eh"] = np.frombuffer(bytes.fromhex(h["eh"]), np.uint8)
        r["version"], r["nentries"] = h["version"], h["nentries"]
        md = bytes.fromhex(h["md"])
        r["md_len"], r["md_off"] = len(md), len(blob)
        blob += md
        alhs.append(bytes.fromhex(h["alh"]))
    return recs, bytes(blob), alhs


def inner_hashes(orc, recs, blob):
    return [orc.tx_header_alh(recs[k], blob)[1] for k in range(len(recs))]
