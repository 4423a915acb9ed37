// gpu_backup_creator.hh -- the zbackup-side binding of libzchunk (include/zchunk.h).
//
// Header-only C++ adapter with BackupCreator's public interface
// (/root/reference/backup_creator.hh:73-89), compiled into zbackup next to
// backup_creator.cc.  ZBackup::backupFromFileHandle (zutils.cc:89-182) keeps its
// read loop and its iterative shrink loop; it only constructs these classes:
//
//   GpuChunkIndex gpuIndex( config, chunkIndex, 0 );            // once per backup
//   GpuBackupCreator backupCreator( gpuIndex, chunkStorageWriter );  // zutils.cc:96
//   ...
//   GpuBackupCreator backupCreator( gpuIndex, chunkStorageWriter );  // zutils.cc:140
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

#include <google/protobuf/io/zero_copy_stream_impl_lite.h>
#include <stdint.h>
#include <string.h>

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

/// The repository's chunk index on the GPU (one libzchunk context)
class GpuChunkIndex: NoCopy, public IndexProcessor
{
  zc_ctx * ctx;
  std::vector< zc_seed > seeds;

public:
  /// flags: ZC_FLAG_SHA1 (the default) is what zbackup needs -- the instruction
  /// stream carries whole ChunkIds (backup_creator.cc:127-141,231-234)
  GpuChunkIndex( Config const & config, ChunkIndex & chunkIndex, int device, uint32_t flags = ZC_FLAG_SHA1 ):
    ctx( 0 )
  {
    zcCheck( zc_create( &ctx, config.GET_STORABLE( chunk, max_size ), device, flags ), 0, "zc_create" );
    chunkIndex.loadIndex( *this );  // every chunk id of every index file -> processChunk
    zcCheck( zc_seed_index( ctx, seeds.data(), seeds.size() ), ctx, "zc_seed_index" );
    std::vector< zc_seed >().swap( seeds );
  }
  ~GpuChunkIndex() { zc_destroy( ctx ); }
  zc_ctx * context() { return ctx; }

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
