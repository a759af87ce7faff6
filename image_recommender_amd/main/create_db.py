"""SQLite schema of the embedding store — mirror of the reference's main/create_db.py.

/root/reference/main/create_db.py:4-131 (ImageDBCreator): ``images(id INTEGER PRIMARY KEY
AUTOINCREMENT, path TEXT UNIQUE)`` plus one ``<type>_vectors(image_id INTEGER PRIMARY KEY
REFERENCES images(id) ON DELETE CASCADE, <type>_vector_blob BLOB)`` table per feature (:49-86);
image paths are POSIX paths relative to the PARENT of the image folder, collected with rglob per
extension in the order .jpg, .jpeg, .png (:97-99), inserted with INSERT OR IGNORE per batch.
Deliberate change: the reference passes Go-style ``_pragma=`` URI parameters that Python's sqlite3
ignores (:37-47); here journal mode / synchronous / busy timeout are applied
as real PRAGMAs.
"""
from __future__ import annotations

import argparse
import sqlite3
from pathlib import Path

VECTOR_TYPES = ("color", "sift", "dreamsim")


class ImageDBCreator:
    def __init__(self, db_path, base_folder, batch_size=8192, timeout=30_000, journal_mode="WAL",
                 synchronous="OFF"):
        dbp = Path(db_path)
        self.db_path = (dbp if dbp.is_absolute() else Path.cwd() / dbp).resolve()
        bf = Path(base_folder)
        self.base_folder = (bf if bf.is_absolute() else Path.cwd() / bf).resolve()
        self.batch_size = batch_size
        self.timeout = timeout
        self.journal_mode = journal_mode
        self.synchronous = synchronous

    def _connect(self):
        conn = sqlite3.connect(self.db_path, timeout=self.timeout / 1000)
        conn.execute(f"PRAGMA journal_mode={self.journal_mode};")
        conn.execute(f"PRAGMA synchronous={self.synchronous};")
        conn.execute("PRAGMA temp_store=MEMORY;")
        conn.execute(f"PRAGMA busy_timeout={int(self.timeout)};")
        return conn

    def create_tables(self):
        with self._connect() as conn:
            create_schema(conn)
        print(f"Tables created in {self.db_path}.")

    def _batch_generator(self):
        exts = (".jpg", ".jpeg", ".png")
        base = Path(self.base_folder)
        all_imgs = [p.relative_to(base.parent).as_posix() for ext in exts
                    for p in base.rglob(f"*{ext}")]
        for i in range(0, len(all_imgs), self.batch_size):
            yield all_imgs[i:i + self.batch_size]

    def process_batches(self):
        self.create_tables()
        with self._connect() as conn:
            for n, batch in enumerate(self._batch_generator(), 1):
                conn.executemany("INSERT OR IGNORE INTO images (path) VALUES (?)",
                                 [(fp,) for fp in batch])
                conn.commit()
                print(f"Batch {n}: inserted {len(batch)} paths.")
        print("All file paths saved to the database.")


def create_schema(conn: sqlite3.Connection, vector_types=VECTOR_TYPES) -> None:
    c = conn.cursor()
    c.execute("CREATE TABLE IF NOT EXISTS images (id INTEGER PRIMARY KEY AUTOINCREMENT, "
              "path TEXT UNIQUE);")
    for t in vector_types:
        c.execute(f"CREATE TABLE IF NOT EXISTS {t}_vectors (image_id INTEGER PRIMARY KEY, "
                  f"{t}_vector_blob BLOB, FOREIGN KEY(image_id) REFERENCES images(id) "
                  f"ON DELETE CASCADE);")
    conn.commit()


def main(argv=None):
    ap = argparse.ArgumentParser(description="Create images.db and register image paths")
    ap.add_argument("--base-folder", default="image_data")
    ap.add_argument("--db-path", default="images.db")
    ap.add_argument("--batch-size", type=int, default=10000)
    a = ap.parse_args(argv)
    ImageDBCreator(a.db_path, a.base_folder, batch_size=a.batch_size).process_batches()


if __name__ == "__main__":
    main()
