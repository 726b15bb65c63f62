"""Extract the mainnet genesis alloc into tests/golden/genesis_alloc.txt.

Run once in the build container (the reference is not present on the GPU box):
    python tests/golden/make_genesis_fixture.py

Input: /root/reference/khipu-eth/src/main/resources/blockchain/default-genesis.json
(the data file GenesisDataLoader.scala:110 loads).  Output: one line per alloc,
"<40-hex address> <decimal balance>", in file order — data only (addresses and
balances), plus the header fields GenesisDataLoader.scala:149-165 uses.
"""
import json
import os

SRC = "/root/reference/khipu-eth/src/main/resources/blockchain/default-genesis.json"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    with open(SRC) as f:
        d = json.load(f)
    with open(os.path.join(HERE, "genesis_alloc.txt"), "w") as f:
        for addr, acc in d["alloc"].items():
            f.write(f"{addr.rjust(40, '0')} {acc['balance']}\n")
    hdr = {k: d[k] for k in ("parentHash", "ommersHash", "coinbase", "difficulty", "gasLimit", "timestamp",
                             "extraData", "mixHash", "nonce")}
    with open(os.path.join(HERE, "genesis_header.json"), "w") as f:
        json.dump(hdr, f, indent=1)
    print(len(d["alloc"]), "allocs")


if __name__ == "__main__":
    main()
