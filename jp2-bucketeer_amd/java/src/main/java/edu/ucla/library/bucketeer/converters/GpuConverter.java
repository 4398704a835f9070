package edu.ucla.library.bucketeer.converters;

import java.io.File;
import java.io.IOException;
import java.net.URLEncoder;
import java.nio.charset.StandardCharsets;
import java.util.concurrent.ArrayBlockingQueue;
import java.util.concurrent.BlockingQueue;
import java.util.concurrent.TimeUnit;
import java.util.concurrent.atomic.AtomicBoolean;

import info.freelibrary.util.Logger;
import info.freelibrary.util.LoggerFactory;

/**
 * A converter that encodes TIFF to JPX on MI355X GPUs through libjp2hip (JNI: libjp2hip_jni.so), in-process,
 * where {@link KakaduConverter} forks kdu_compress (KakaduConverter.java:55-77). Same recipe, same output name
 * (<tmp>/jp2hip/URL-encoded id + ".jpx"), every failure an {@link IOException} (AbstractConverter.java:33-35).
 * Thread-safe: each {@link #convert} borrows one native context (one GPU stream) from a pool.
 */
public class GpuConverter extends AbstractConverter implements Converter, AutoCloseable {

    private static final Logger LOGGER = LoggerFactory.getLogger(GpuConverter.class, "bucketeer_messages");

    /**
     * Contexts (images in flight) per GPU: system property; default 0 = as many as fit 75 % of the device's free
     * memory at 8 GiB each, at most 16 (hipMemGetInfo through the glue; DESIGN.md 3 "Footprint").
     */
    static final String CONTEXTS_PER_GPU = "bucketeer.gpu.contexts";

    /** Images of at least this many pixels are tile-split across every GPU (C5 map scans). */
    static final String SPLIT_MIN_PIXELS = "bucketeer.gpu.split.min.pixels";

    private static final File TMP_DIR = new File(System.getProperty("java.io.tmpdir"), "jp2hip");

    private static final boolean LOADED = load();

    /** {split context or 0, pooled contexts...}: what close() releases */
    private final long[] myHandles;

    /** pooled contexts; a convert() borrows one */
    private final BlockingQueue<Long> myContexts;

    private final long mySplitMinPixels;

    /** non-null: why this converter cannot encode; every convert() throws IOException */
    private final String myUnavailable;

    /** set once by close(); read without a lock by every convert() and by waiting borrowers */
    private final AtomicBoolean myClosed = new AtomicBoolean();

    /** serialises split encodes with each other (and with close()), never with pooled conversions */
    private final Object mySplitLock = new Object();

    /** how often a borrower waiting for a context re-checks myClosed */
    private static final long BORROW_POLL_MS = 100;

    /**
     * Package-private, like KakaduConverter's (KakaduConverter.java:48). The native side either creates every
     * context or none: a failure part-way releases what it created before the IOException reaches here.
     */
    GpuConverter() throws IOException {
        if (!TMP_DIR.exists() && !TMP_DIR.mkdirs()) {
            throw new IOException("Cannot create " + TMP_DIR);
        }
        if (!LOADED) {
            throw new IOException("libjp2hip_jni not loadable");
        }
        final int perGpu = Math.max(0, Integer.getInteger(CONTEXTS_PER_GPU, 0)); // 0: from device memory
        mySplitMinPixels = Long.getLong(SPLIT_MIN_PIXELS, 256_000_000L);
        myHandles = nativeOpen(perGpu, mySplitMinPixels); // throws IOException, nothing allocated then
        myContexts = new ArrayBlockingQueue<>(Math.max(1, myHandles.length - 1));
        for (int index = 1; index < myHandles.length; index++) {
            myContexts.add(myHandles[index]);
        }
        myUnavailable = null;
        final String advice = nativeEnvCheck(); // GPU_MAX_HW_QUEUES
        if (!advice.isEmpty()) {
            LOGGER.warn("libjp2hip: " + advice);
        }
    }

    private GpuConverter(final String aReason) {
        myHandles = new long[0];
        myContexts = new ArrayBlockingQueue<>(1);
        mySplitMinPixels = Long.MAX_VALUE;
        myUnavailable = aReason;
    }

    /** A converter that fails every conversion with IOException (never a runtime exception). */
    static GpuConverter unavailable(final String aReason) {
        return new GpuConverter(aReason);
    }

    static boolean isAvailable() {
        return LOADED && nativeProbe();
    }

    @Override
    public File convert(final String aID, final File aTIFF, final Conversion aConversion)
            throws IOException, InterruptedException {
        if (myUnavailable != null) {
            throw new IOException("Failed to convert TIFF to JP2: " + aID + ": " + myUnavailable);
        }
        final File jpx = new File(TMP_DIR, URLEncoder.encode(aID, StandardCharsets.UTF_8.toString()) + ".jpx");
        final byte[] tiff = aTIFF.getAbsolutePath().getBytes(StandardCharsets.UTF_8);
        final byte[] out = jpx.getAbsolutePath().getBytes(StandardCharsets.UTF_8);
        final String error;
        final long split = myHandles[0];
        if (myClosed.get()) {
            throw new IOException("Failed to convert TIFF to JP2: " + aID + ": converter closed");
        }
        if (split != 0 && nativeTiffPixels(tiff) >= mySplitMinPixels) {
            synchronized (mySplitLock) { // one oversized image at a time holds every GPU
                if (myClosed.get()) {
                    throw new IOException("Failed to convert TIFF to JP2: " + aID + ": converter closed");
                }
                error = nativeEncodeFile(split, tiff, out, aConversion.ordinal());
            }
        } else {
            final long ctx = borrow(aID);
            try {
                error = nativeEncodeFile(ctx, tiff, out, aConversion.ordinal()); // LOSSY=0, LOSSLESS=1
            } finally {
                myContexts.put(ctx);
            }
        }
        if (error != null) {
            throw new IOException("Failed to convert TIFF to JP2: " + aID + ": " + error);
        }
        return jpx;
    }

    /**
     * A pooled context, or IOException once close() has begun: a waiter re-checks myClosed every
     * BORROW_POLL_MS, so it never blocks on a pool that close() is draining.
     */
    private long borrow(final String aID) throws IOException, InterruptedException {
        while (true) {
            final Long ctx = myContexts.poll(BORROW_POLL_MS, TimeUnit.MILLISECONDS);
            if (myClosed.get()) {
                if (ctx != null) {
                    myContexts.put(ctx); // close() is counting them back
                }
                throw new IOException("Failed to convert TIFF to JP2: " + aID + ": converter closed");
            }
            if (ctx != null) {
                return ctx;
            }
        }
    }

    /**
     * Releases the GPU contexts once every borrowed one is back (conversions in progress finish first). Later
     * conversions fail with IOException.
     */
    @Override
    public void close() throws InterruptedException {
        if (!myClosed.compareAndSet(false, true) || myHandles.length == 0) {
            return;
        }
        for (int index = 1; index < myHandles.length; index++) {
            myContexts.take(); // waits for conversions that hold one; waiting borrowers give up
        }
        synchronized (mySplitLock) { // a split encode in progress finishes first
            nativeClose(myHandles);
        }
    }

    @Override
    public String getExecutable() {
        return "libjp2hip";
    }

    private static boolean load() {
        try {
            System.loadLibrary("jp2hip_jni"); // links libjp2hip.so
            return true;
        } catch (final UnsatisfiedLinkError details) {
            return false;
        }
    }

    private static native boolean nativeProbe();

    private static native String nativeEnvCheck();

    /** @return {split context (0 on one GPU), pooled contexts...}; IOException leaves nothing allocated */
    private static native long[] nativeOpen(int aPerGpu, long aSplitMinPixels) throws IOException;

    private static native void nativeClose(long[] aHandles);

    /** @return width x height from the TIFF header, or -1 (the encode then reports the error) */
    private static native long nativeTiffPixels(byte[] aTiff);

    /** @return null on success, else jp2hip_last_error() of the calling thread */
    private static native String nativeEncodeFile(long aCtx, byte[] aTiff, byte[] aOut, int aConversion);
}
