// pqwrite.cpp — parquet writer with column-parallel encoding (libmdpq.so).
//
// The reference writes every parquet file through pyarrow's write_table
// (/root/reference/metadamage/io.py:79-83).  pyarrow encodes and compresses the
// columns of a row group one after another on the calling thread: the counts
// table of a 100k-taxon file (2.8 M rows x 30 columns) takes ~0.45 s of one
// core, the largest host stage of the streamed C5 pipeline.
// This writes the same table -- same schema, same key-value metadata (the
// "metadamage" config and pandas' own), the stored Arrow schema, format 2.6,
// snappy pages, dictionaries and statistics on the categorical columns only --
// through libparquet with ArrowWriterProperties::use_threads, so the column
// chunks of a row group are encoded on Arrow's CPU pool in parallel.  The file
// reads back identical with any pyarrow (tests/test_counts.py).
//
// Round 6: the page compression (snappy or none) and the columns that carry
// statistics are parameters: the streamed pipeline writes its large tables
// (the counts cache, the per-position predictions) uncompressed with
// statistics on tax_id only -- half the encoding CPU of snappy pages on the
// count columns, which compress ~2x at best.
//
// C ABI (ctypes):
//   mdpq_unwrap(PyObject* table) -> handle   (call with the GIL held: PyDLL)
//   mdpq_write(handle, path, dict_cols, n_dict, stat_cols, n_stat, snappy,
//              row_group_rows) -> 0 / -1     (GIL released: CDLL; frees handle)
//   mdpq_free(handle), mdpq_last_error()
#include <Python.h>

#include <arrow/api.h>
#include <arrow/io/file.h>
#include <arrow/python/pyarrow.h>
#include <parquet/arrow/writer.h>
#include <parquet/properties.h>

#include <cstring>
#include <memory>
#include <string>

namespace {
thread_local std::string g_err;

struct Handle {
  std::shared_ptr<arrow::Table> table;
};
}  // namespace

extern "C" {

const char* mdpq_last_error(void) { return g_err.c_str(); }

void* mdpq_unwrap(PyObject* obj) {
  static bool imported = false;
  if (!imported) {
    if (arrow::py::import_pyarrow() != 0) {
      g_err = "import_pyarrow failed";
      return nullptr;
    }
    imported = true;
  }
  auto r = arrow::py::unwrap_table(obj);
  if (!r.ok()) {
    g_err = r.status().ToString();
    return nullptr;
  }
  return new Handle{*r};
}

void mdpq_free(void* h) { delete static_cast<Handle*>(h); }

int mdpq_write(void* h, const char* path, const char** dict_cols, int n_dict, const char** stat_cols, int n_stat,
               int snappy, int64_t row_group_rows) {
  std::unique_ptr<Handle> hd(static_cast<Handle*>(h));
  if (!hd || !hd->table || !path) {
    g_err = "bad arguments";
    return -1;
  }
  parquet::WriterProperties::Builder wb;
  wb.version(parquet::ParquetVersion::PARQUET_2_6);
  wb.compression(snappy ? parquet::Compression::SNAPPY : parquet::Compression::UNCOMPRESSED);
  wb.disable_dictionary();
  wb.disable_statistics();
  for (int i = 0; i < n_dict; ++i) wb.enable_dictionary(dict_cols[i]);
  for (int i = 0; i < n_stat; ++i) wb.enable_statistics(stat_cols[i]);
  parquet::ArrowWriterProperties::Builder ab;
  ab.set_use_threads(true);
  ab.store_schema();
  auto out = arrow::io::FileOutputStream::Open(path);
  if (!out.ok()) {
    g_err = out.status().ToString();
    return -1;
  }
  const int64_t rg = row_group_rows > 0 ? row_group_rows : parquet::DEFAULT_MAX_ROW_GROUP_LENGTH;
  wb.max_row_group_length(rg);
  // buffered row groups: WriteRecordBatch encodes the batch's columns in
  // parallel (use_threads); one batch per row group, as write_table cuts them
  auto run = [&]() -> arrow::Status {
    ARROW_ASSIGN_OR_RAISE(auto w, parquet::arrow::FileWriter::Open(*hd->table->schema(), arrow::default_memory_pool(),
                                                                   *out, wb.build(), ab.build()));
    arrow::TableBatchReader rd(*hd->table);
    rd.set_chunksize(rg);
    std::shared_ptr<arrow::RecordBatch> batch;
    // one buffered row group: the writer closes it and opens the next at
    // max_row_group_length, so the row groups are write_table's
    ARROW_RETURN_NOT_OK(w->NewBufferedRowGroup());
    while (true) {
      ARROW_RETURN_NOT_OK(rd.ReadNext(&batch));
      if (!batch) break;
      ARROW_RETURN_NOT_OK(w->WriteRecordBatch(*batch));
    }
    ARROW_RETURN_NOT_OK(w->Close());
    return (*out)->Close();
  };
  const arrow::Status st = run();
  if (!st.ok()) {
    g_err = st.ToString();
    return -1;
  }
  return 0;
}

}  // extern "C"
