// gpu_backup_creator.hh -- the zbackup-side binding of libzchunk (include/zchunk.h).
//
// Header-only C++ adapter with BackupCreator's public interface
// (/root/reference/backup_creator.hh:73-89), compiled into zbackup next to
// backup_creator.cc.  ZBackup::backupFromFileHandle (zutils.cc:89-182) keeps its
// read loop and its iterative shrink loop; it only constructs these classes:
//
//   GpuChunkIndex gpuIndex( config, chunkIndex, 0, ZC_FLAG_SHA1, metaDir );  // once per backup
//   GpuBackupCreator backupCreator( gpuIndex, chunkStorageWriter );  // zutils.cc:96
//   ...
//   GpuBackupCreator backupCreator( gpuIndex, chunkStorageWriter );  // zutils.cc:140
//   ...
//   chunkStorageWriter.commit();                                     // zutils.cc:175
//   gpuIndex.saveChunkMeta( metaDir );   // metaDir = Dir::addPath( dir, "zchunk" )
//
// GpuChunkIndex is the device-side probe set: one libzchunk context, seeded
// with every chunk id of the repository's index files (ChunkIndex::loadIndex
// driving this class as its IndexProcessor, chunk_index.cc:26-79).  Every
// GpuBackupCreator on it is one stream on that context (zc_reset), so a shrink
// pass matches the chunks the passes before it wrote, as the reference's
// passes share one ChunkIndex that Writer::add grows (chunk_storage.cc:31-46).
//
// Records are taken as they are cut (zc_take_records, during handleMoreData):
// a NEW chunk goes to Writer::add with its bytes, every record to the
// instruction stream (Message::serialize, message.cc:16-23), exactly as
// saveChunkToSave / addChunkIfMatched / outputInstruction do
// (backup_creator.cc:110-145,242-273).  Errors become exceptions, as the
// reference's DEF_EX / CHECK paths are.
#ifndef GPU_BACKUP_CREATOR_HH_INCLUDED
#define GPU_BACKUP_CREATOR_HH_INCLUDED

#include <dirent.h>
#include <google/protobuf/io/zero_copy_stream_impl_lite.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "chunk_id.hh"
#include "chunk_index.hh"
#include "chunk_storage.hh"
#include "config.hh"
#include "message.hh"
#include "nocopy.hh"
#include "sptr.hh"
#include "zbackup.pb.h"
#include "zchunk.h"

inline void zcCheck( int rc, zc_ctx * ctx, char const * what )
{
  if ( rc != ZC_OK )
    throw std::runtime_error( std::string( what ) + ": " + ( ctx ? zc_last_error( ctx ) : "libzchunk" ) );
}

/// The content-anchor metadata of a repository's chunks (zc_chunk_meta, ABI 5),
/// kept in files of its own beside the index -- "<repo>/zchunk/<sha256 hex>" --
/// and never inside index/ or bundles/, whose formats stay zbackup's.  One
/// file per backup, written at the end of the backup next to the index file
/// Writer::commit moves into place (chunk_storage.cc:61-90); a new process
/// reads every file and seeds the ids ChunkIndex::loadIndex reports together
/// with the entries that match them by full ChunkId.  The metadata is a pure
/// function of a chunk's bytes, so it never goes stale: entries of chunks a gc
/// removed are simply never joined to an id, and a file that is damaged or of
/// another anchor definition only costs speed (those ids are screened by key),
/// never a different backup.
///
/// File: "ZCMETA01", LE32 record size (48), LE32 0, LE64 count, count records,
/// then the SHA-256 of everything before it (zc_sha256_*); written to a
/// temporary name and renamed, as tmp_mgr.cc:16-24 does for zbackup's files.
class GpuChunkMetaSidecar
{
  static void sha256( std::string const & data, unsigned char out[ 32 ] )
  {
    zc_sha256 * h = 0;
    if ( zc_sha256_create( &h ) != ZC_OK )
      throw std::runtime_error( "zc_sha256_create" );
    zc_sha256_add( h, data.data(), data.size() );
    zc_sha256_finish( h, out );
    zc_sha256_destroy( h );
  }

public:
  /// the entries of one file; false (and nothing added) if it is not a valid one
  static bool read( std::string const & path, std::vector< zc_chunk_meta > & out )
  {
    FILE * f = fopen( path.c_str(), "rb" );
    if ( !f )
      return false;
    std::string data;
    char buf[ 65536 ];
    size_t rd;
    while ( ( rd = fread( buf, 1, sizeof( buf ), f ) ) > 0 )
      data.append( buf, rd );
    fclose( f );
    if ( data.size() < 24 + 32 || data.compare( 0, 8, "ZCMETA01" ) != 0 )
      return false;
    uint32_t recSize;
    uint64_t count;
    memcpy( &recSize, data.data() + 8, 4 );
    memcpy( &count, data.data() + 16, 8 );
    if ( recSize != sizeof( zc_chunk_meta ) || count > ( data.size() - 56 ) / recSize ||
         data.size() != 24 + count * recSize + 32 )
      return false;
    unsigned char want[ 32 ];
    sha256( data.substr( 0, data.size() - 32 ), want );
    if ( memcmp( want, data.data() + data.size() - 32, 32 ) != 0 )
      return false;
    size_t at = out.size();
    out.resize( at + count );
    memcpy( &out[ at ], data.data() + 24, count * recSize );
    return true;
  }

  /// every valid file of dir (a missing dir: none)
  static void readDir( std::string const & dir, std::vector< zc_chunk_meta > & out )
  {
    DIR * d = opendir( dir.c_str() );
    if ( !d )
      return;
    while ( struct dirent * e = readdir( d ) )
    {
      std::string name( e->d_name );
      if ( name.size() == 64 && name.find_first_not_of( "0123456789abcdef" ) == std::string::npos )
        read( dir + "/" + name, out );
    }
    closedir( d );
  }

  /// the metadata of the chunks ctx's streams added, as one new file of dir
  /// (made if missing); returns its path, or "" when there is nothing to write
  static std::string write( std::string const & dir, zc_ctx * ctx )
  {
    size_t n = 0;
    zc_export_chunk_meta( ctx, 0, 0, &n );
    if ( !n )
      return std::string();
    std::vector< zc_chunk_meta > meta( n );
    zcCheck( zc_export_chunk_meta( ctx, meta.data(), meta.size(), &n ), ctx, "zc_export_chunk_meta" );
    std::string data( "ZCMETA01", 8 );
    uint32_t words[ 2 ] = { (uint32_t)sizeof( zc_chunk_meta ), 0 };
    uint64_t count = n;
    data.append( (char const *)words, 8 );
    data.append( (char const *)&count, 8 );
    data.append( (char const *)meta.data(), n * sizeof( zc_chunk_meta ) );
    unsigned char sum[ 32 ];
    sha256( data, sum );
    data.append( (char const *)sum, 32 );
    char hex[ 65 ];
    for ( int i = 0; i < 32; ++i )
      snprintf( hex + 2 * i, 3, "%02x", sum[ i ] );
    mkdir( dir.c_str(), 0755 );
    std::string path = dir + "/" + hex, tmp = path + ".tmp";
    FILE * f = fopen( tmp.c_str(), "wb" );
    if ( !f || fwrite( data.data(), 1, data.size(), f ) != data.size() || fflush( f ) != 0 ||
         fsync( fileno( f ) ) != 0 )
    {
      if ( f )
        fclose( f );
      unlink( tmp.c_str() );
      throw std::runtime_error( "chunk metadata: cannot write " + tmp );
    }
    fclose( f );
    if ( rename( tmp.c_str(), path.c_str() ) != 0 )
    {
      unlink( tmp.c_str() );
      throw std::runtime_error( "chunk metadata: cannot rename " + tmp );
    }
    return path;
  }
};

/// The repository's chunk index on the GPU (one libzchunk context)
class GpuChunkIndex: NoCopy, public IndexProcessor
{
  zc_ctx * ctx;
  std::vector< zc_seed > seeds;

public:
  /// flags: ZC_FLAG_SHA1 (the default) is what zbackup needs -- the instruction
  /// stream carries whole ChunkIds (backup_creator.cc:127-141,231-234).
  /// metaDir: the repository's chunk-metadata directory (GpuChunkMetaSidecar),
  /// or "" to seed the ids alone
  GpuChunkIndex( Config const & config, ChunkIndex & chunkIndex, int device, uint32_t flags = ZC_FLAG_SHA1,
                 std::string const & metaDir = std::string() ):
    ctx( 0 )
  {
    zcCheck( zc_create( &ctx, config.GET_STORABLE( chunk, max_size ), device, flags ), 0, "zc_create" );
    // the feed window's buffers (pinned host mirror + HBM, ~0.3 s to pin 1 GiB)
    // are made on a helper thread while the index loads
    zcCheck( zc_set_window( ctx, zc_get_window( ctx ) ), ctx, "zc_set_window" );
    chunkIndex.loadIndex( *this );  // every chunk id of every index file -> processChunk
    std::vector< zc_chunk_meta > meta;
    if ( !metaDir.empty() )
      GpuChunkMetaSidecar::readDir( metaDir, meta );
    if ( meta.empty() )
      zcCheck( zc_seed_index( ctx, seeds.data(), seeds.size() ), ctx, "zc_seed_index" );
    else
      zcCheck( zc_seed_index_meta( ctx, seeds.data(), seeds.size(), meta.data(), meta.size() ), ctx,
               "zc_seed_index_meta" );
    std::vector< zc_seed >().swap( seeds );
  }
  ~GpuChunkIndex() { zc_destroy( ctx ); }
  zc_ctx * context() { return ctx; }

  /// after chunkStorageWriter.commit() (zutils.cc:175): the metadata of the
  /// chunks this backup wrote, as a new file of metaDir
  std::string saveChunkMeta( std::string const & metaDir ) { return GpuChunkMetaSidecar::write( metaDir, ctx ); }

  // IndexProcessor (chunk_index.hh:47-55)
  void startIndex( string const & ) {}
  void startBundle( Bundle::Id const & ) {}
  void processChunk( ChunkId const & id, uint32_t size )
  {
    zc_seed s;
    memcpy( s.sha1, id.cryptoHash, sizeof( s.sha1 ) );
    s.rolling = id.rollingHash;
    s.size = size;
    s.reserved = 0;
    seeds.push_back( s );
  }
  void finishBundle( Bundle::Id const &, BundleInfo const & ) {}
  void finishIndex( string const & ) {}
};

/// BackupCreator's interface (backup_creator.hh:73-89) over libzchunk
class GpuBackupCreator: NoCopy
{
  zc_ctx * ctx;
  ChunkStorage::Writer & chunkStorageWriter;
  string backupData;
  sptr< google::protobuf::io::StringOutputStream > backupDataStream;
  std::vector< zc_record > records;
  string bytes;

  void take( zc_record const & r )
  {
    BackupInstruction instr;
    if ( r.kind == ZC_BYTES )  // backup_creator.cc:114-121
    {
      bytes.resize( r.size );
      zcCheck( zc_read_stream( ctx, r.offset, r.size, &bytes[ 0 ] ), ctx, "zc_read_stream" );
      instr.set_bytes_to_emit( bytes );
    }
    else
    {
      ChunkId id;
      memcpy( id.cryptoHash, r.sha1, sizeof( id.cryptoHash ) );
      id.rollingHash = r.rolling;
      if ( r.kind == ZC_CHUNK_NEW )  // saveChunkToSave: backup_creator.cc:124-139
      {
        // the chunk's bytes straight from the feed window's host mirror (no
        // copy); a device-resident stream's are copied out
        void const * data = zc_stream_data( ctx, r.offset, r.size );
        if ( !data )
        {
          bytes.resize( r.size );
          zcCheck( zc_read_stream( ctx, r.offset, r.size, &bytes[ 0 ] ), ctx, "zc_read_stream" );
          data = bytes.data();
        }
        chunkStorageWriter.add( id, data, r.size );
      }
      instr.set_chunk_to_emit( id.toBlob() );
    }
    Message::serialize( instr, *backupDataStream );  // outputInstruction: backup_creator.cc:267-273
  }

  // the records cut so far, in stream order; their bytes are readable until
  // the next feed call
  void drain()
  {
    for ( ; ; )
    {
      records.resize( 4096 );
      size_t got = 0;
      zcCheck( zc_take_records( ctx, records.data(), records.size(), &got ), ctx, "zc_take_records" );
      for ( size_t i = 0; i < got; ++i )
        take( records[ i ] );
      if ( got < records.size() )
        break;
    }
  }

public:
  GpuBackupCreator( GpuChunkIndex & index, ChunkStorage::Writer & writer ):
    ctx( index.context() ), chunkStorageWriter( writer ),
    backupDataStream( new google::protobuf::io::StringOutputStream( &backupData ) )
  {
    zcCheck( zc_reset( ctx ), ctx, "zc_reset" );  // a new stream on the shared index
  }

  void * getInputBuffer()  // backup_creator.cc:40-43
  {
    void * p = zc_get_input_buffer( ctx );
    if ( !p )
      zcCheck( ZC_ERR_STATE, ctx, "getInputBuffer" );
    return p;
  }

  size_t getInputBufferSize()  // backup_creator.cc:45-54
  {
    size_t n = zc_get_input_buffer_size( ctx );
    if ( !n )
      zcCheck( ZC_ERR_STATE, ctx, "getInputBufferSize" );
    return n;
  }

  void handleMoreData( unsigned added )  // backup_creator.cc:56-108
  {
    zcCheck( zc_handle_more_data( ctx, added ), ctx, "handleMoreData" );
    drain();
  }

  void finish()  // backup_creator.cc:147-172
  {
    zcCheck( zc_finish( ctx ), ctx, "finish" );
    drain();
  }

  void getBackupData( string & str )  // backup_creator.cc:275-280
  {
    if ( !backupDataStream.get() )
      throw std::logic_error( "getBackupData() called twice" );
    backupDataStream.reset();
    str.swap( backupData );
  }
};

/// lzo1x_1 of finished bundles on the GPU, for Bundle::Creator::write
/// (bundle.cc:96-155) when the selected compression is "lzo1x_1": the framed
/// bytes equal what LZO1X_1_Encoder writes (compression.cc:435-466, 586-606),
/// so the encoder loop there becomes
///
///   string framed;
///   gpuLzo.compress( payload, framed );    // one payload, or compressAll for a batch
///   os.write( framed.data(), framed.size() );
///
/// (EncryptedFile::OutputStream::write, as bundle.cc:84 uses it), followed by the
/// os.writeAdler32() the reference already does.
///
/// Bundle::Creator::write runs on detached compressor threads, several at a time
/// (chunk_storage.cc:133-141,175), while the main thread feeds the backup stream
/// through GpuChunkIndex's context.  So this class never touches that context:
/// it keeps a pool of contexts of its own, one per compressor thread that is
/// inside compress() at the moment (made on first need, reused after), and each
/// call runs on a context no other thread is using.  (libzchunk also serializes
/// the calls on one context with a per-context lock, so sharing one would be
/// safe, only not concurrent.)
class GpuLzoBundleCompressor: NoCopy
{
  int device;
  std::mutex poolMutex;
  std::vector< zc_ctx * > idle, all;

  zc_ctx * acquire()
  {
    std::lock_guard< std::mutex > lock( poolMutex );
    if ( !idle.empty() )
    {
      zc_ctx * c = idle.back();
      idle.pop_back();
      return c;
    }
    zc_ctx * c = 0;
    zcCheck( zc_create( &c, 65536, device, 0 ), 0, "zc_create" );
    all.push_back( c );
    return c;
  }

  void release( zc_ctx * c )
  {
    std::lock_guard< std::mutex > lock( poolMutex );
    idle.push_back( c );
  }

public:
  explicit GpuLzoBundleCompressor( int device_ = 0 ): device( device_ ) {}
  ~GpuLzoBundleCompressor()
  {
    for ( size_t i = 0; i < all.size(); ++i )
      zc_destroy( all[ i ] );
  }

  void compress( string const & payload, string & framed )
  {
    std::vector< string const * > one( 1, &payload );
    std::vector< string > out;
    compressAll( one, out );
    framed.swap( out[ 0 ] );
  }

  /// several finished bundles in one device call (Writer::finishCurrentBundle
  /// can queue them instead of starting a compressor thread per bundle)
  void compressAll( std::vector< string const * > const & payloads, std::vector< string > & framed )
  {
    size_t n = payloads.size();
    std::vector< uint64_t > payOff( n ), paySize( n ), outOff( n ), outSize( n );
    string in, out;
    uint64_t inPos = 0, outPos = 0;
    for ( size_t i = 0; i < n; ++i )
    {
      payOff[ i ] = inPos;
      paySize[ i ] = payloads[ i ]->size();
      inPos += paySize[ i ];
      outOff[ i ] = outPos;
      outPos += zc_lzo_capacity( paySize[ i ] );
    }
    in.reserve( inPos );
    for ( size_t i = 0; i < n; ++i )
      in += *payloads[ i ];
    out.resize( outPos ? outPos : 1 );
    zc_ctx * ctx = acquire();
    int rc = zc_lzo_compress_host( ctx, in.data(), payOff.data(), paySize.data(), n, &out[ 0 ], outOff.data(),
                                   outSize.data() );
    string err = rc == ZC_OK ? string() : string( zc_last_error( ctx ) );
    release( ctx );
    if ( rc != ZC_OK )
      throw std::runtime_error( "zc_lzo_compress_host: " + err );
    framed.resize( n );
    for ( size_t i = 0; i < n; ++i )
      framed[ i ].assign( out, outOff[ i ], outSize[ i ] );
  }
};

#endif
